"""Meta items (Dataset3.meta_items) and diff_meta against the reference's own outputs
(tests/golden, written by the reference's ``RichBaseDataset.diff_meta`` over its test repositories
and the crafted ``meta_edits`` history: title, description, CRS definitions re-spaced / added /
nested / removed, the metadata.xml attachment, a schema.json that only changes its formatting, and
non-standard meta files)."""
import pytest

from fixtures import DIFF_FIXTURES, load
from kart_amd import deltas, meta


@pytest.mark.parametrize("name", DIFF_FIXTURES)
def test_diff_meta_golden(name):
    fx = load(name)
    for case in fx.cases("diff2"):
        old = meta.meta_items(fx.meta_files(case["base"]), fx.attachments(case["base"])) if fx.n(case["base"]) or \
            fx.meta["sides"][case["base"]]["schema"] else {}
        new = meta.meta_items(fx.meta_files(case["target"]), fx.attachments(case["target"])) if fx.n(case["target"]) or \
            fx.meta["sides"][case["target"]]["schema"] else {}
        dd = deltas.DeltaDiff.diff_dicts(old, new)
        got = sorted([k, d.old_value, d.new_value] for k, d in dd.items())
        assert got == case["meta"], (name, case["base"], case["target"])


def test_meta_items_standard_only():
    fx = load("meta_edits")
    items = meta.meta_items(fx.meta_files("c0"), fx.attachments("c0"))
    assert set(items) == {"title", "schema.json", "metadata.xml", "crs/EPSG:4326.wkt"}  # custom.json is not one
    assert items["metadata.xml"].startswith("<gmd:MD_Metadata>")
    assert meta.meta_items({}, {"metadata.xml": b"x"}) == {}  # no meta tree: no items at all


def test_normalise_wkt_golden():
    """normalise_wkt == the reference's crs_util.normalise_wkt on crafted WKT (tests/golden/wkt.json:
    whitespace, nesting, error characters, unbalanced brackets, newlines, a BOM, non-ASCII)"""
    import json
    import os

    from fixtures import GOLDEN

    with open(os.path.join(GOLDEN, "wkt.json")) as f:
        cases = json.load(f)
    assert len(cases) >= 15
    for wkt, want in cases:
        assert meta.normalise_wkt(wkt) == want, wkt
    assert meta.normalise_wkt("") == "" and meta.normalise_wkt(None) is None


def test_normalise_column_dicts():
    cols = [{"name": "fid", "id": "a", "dataType": "integer", "primaryKeyIndex": 0, "size": 64},
            {"length": None, "id": "b", "dataType": "text", "name": "n", "primaryKeyIndex": None}]
    assert meta.normalise_column_dicts(cols) == [
        {"id": "a", "name": "fid", "dataType": "integer", "primaryKeyIndex": 0, "size": 64},
        {"id": "b", "name": "n", "dataType": "text"}]
