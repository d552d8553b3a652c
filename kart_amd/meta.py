"""A dataset version's meta items, as Dataset3.meta_items yields them (the input of diff_meta).

Reference: ``BaseDataset.meta_items`` (kart/base_dataset.py:339-355), ``Dataset3.get_meta_item`` and
``crs_definitions`` (kart/dataset3.py:127-160), ``META_ITEM_NAMES`` / ``ATTACHMENT_META_ITEMS``
(kart/meta_items.py:4-14), ``Schema.normalise_column_dicts`` (kart/schema.py:264-266,
``ColumnSchema.from_dict`` / ``to_dict`` :158-175) and ``crs_util.normalise_wkt``
(kart/crs_util.py:204-209, the pretty-printing ``WKTLexer`` of kart/wkt_lexer.py).

``diff_meta`` then is ``DeltaDiff.diff_dicts(old.meta_items(), new.meta_items())``
(kart/rich_base_dataset.py:183-195): the standard items (title, description, the normalised
schema.json, the ``metadata.xml`` attachment kept next to ``.table-dataset``) when non-empty, plus
every CRS definition under ``meta/crs/`` keyed ``crs/<its name minus 4 characters>.wkt``.  Legends,
path-structure.json and any other file in the meta tree are not items.
"""
import json
import re

META_ITEM_NAMES = ("title", "description", "schema.json", "metadata.xml")
ATTACHMENT_META_ITEMS = ("metadata.xml",)
CRS_DIR = "crs/"


def ensure_text(data):
    return data.decode("utf8") if isinstance(data, (bytes, bytearray, memoryview)) else data


def normalise_column_dicts(column_dicts):
    """Schema.normalise_column_dicts: every column as ColumnSchema.to_dict writes it — id, name,
    dataType, primaryKeyIndex when set, then its other attributes in their order, None-valued ones
    dropped (and ColumnSchema's own checks: an unknown data type is refused)"""
    out = []
    for d in column_dicts:
        d = dict(d)
        col = {"id": d.pop("id"), "name": d.pop("name"), "dataType": d.pop("dataType")}
        if col["dataType"] not in _DATA_TYPES:
            raise AssertionError(col["dataType"])
        pk = d.pop("primaryKeyIndex", None)
        if pk is not None:
            col["primaryKeyIndex"] = pk
        col.update((k, v) for k, v in d.items() if v is not None)
        out.append(col)
    return out


_DATA_TYPES = {"boolean", "blob", "date", "float", "geometry", "integer", "interval", "numeric", "text", "time",
               "timestamp"}


# ---- WKT normalisation ------------------------------------------------------------------------
# The reference's WKT lexer tokenises WKT 1 with a small state machine (a value is a number, a
# quoted string, a keyword or a bracketed list; a list holds values separated by commas) and the
# pretty-printer drops the original whitespace and re-emits the tokens: a keyword that follows a
# comma and opens a bracket starts a new line, indented four spaces per open keyword, any other
# token after a comma gets one space, and the text ends with a newline.  Restated here token for
# token, including what the lexer does with characters it cannot place (single-character error
# tokens, printed as they are).
_WS = re.compile(r"\s+")
_FLOAT = re.compile(r"-?(0|[1-9]\d*)(\.\d+[eE](\+|-)?\d+|[eE](\+|-)?\d+|\.\d+)")
_INT = re.compile(r"-?(0|[1-9]\d*)")
_STR = re.compile(r'"(""|[^"])*"')
_KEYWORD = re.compile(r"\w(\w|\d|_)*")
_OPEN = re.compile(r"(\[|\()")
_COMMA = re.compile(r",")
_CLOSE = re.compile(r"(\]|\))")
WS, NUM, STR, KEYWORD, OPEN, COMMA, CLOSE, ERROR = range(8)


def _tokens(text):
    """(kind, text) tokens of WKT, whitespace included"""
    # the lexer's input preparation: newlines normalised, leading/trailing newlines stripped, one
    # trailing newline ensured
    if text.startswith("﻿"):
        text = text[1:]
    text = text.replace("\r\n", "\n").replace("\r", "\n").strip("\n")
    if not text.endswith("\n"):
        text += "\n"
    value_rules = [(_WS, WS), (_FLOAT, NUM), (_INT, NUM), (_STR, STR), (_KEYWORD, KEYWORD), (_OPEN, OPEN)]
    list_rules = value_rules + [(_COMMA, COMMA), (_CLOSE, CLOSE)]
    depth, pos, out = 0, 0, []
    while pos < len(text):
        for rx, kind in (list_rules if depth else value_rules):
            m = rx.match(text, pos)
            if m and m.end() > pos:
                out.append((kind, m.group(0)))
                pos = m.end()
                if kind == OPEN:
                    depth += 1
                elif kind == CLOSE:
                    depth -= 1
                break
        else:
            if text[pos] == "\n":  # at an unmatched newline the lexer returns to its start state
                depth = 0
                out.append((WS, "\n"))
            else:
                out.append((ERROR, text[pos]))
            pos += 1
    return out


def normalise_wkt(wkt):
    """crs_util.normalise_wkt: the WKT's tokens re-spaced as the reference's pretty-printer does"""
    if not wkt:
        return wkt
    toks = [t for t in _tokens(wkt) if t[0] != WS]
    pad = [(WS, "")]
    seq = pad + toks + pad
    out, indent = [], 0
    for i in range(1, len(seq) - 1) if len(seq) >= 3 else ():
        prev, cur, nxt = seq[i - 1], seq[i], seq[i + 1]
        if prev[0] == COMMA:
            if cur[0] == KEYWORD and nxt[0] == OPEN:
                indent += 1
                out.append("\n" + "    " * indent)
            else:
                out.append(" ")
        if cur[0] == CLOSE:
            indent = max(indent - 1, 0)
        out.append(cur[1])
    out.append("\n")
    return "".join(out)


# ---- the items ---------------------------------------------------------------------------------
def meta_item_value(name, data):
    """Dataset3.get_meta_item's decoding of one item's bytes"""
    if data is None:
        return None
    if name.endswith("schema.json"):
        return normalise_column_dicts(json.loads(data))
    if name.endswith(".json"):
        return json.loads(data)
    if name.endswith(".wkt"):
        return normalise_wkt(ensure_text(data))
    return ensure_text(data)


def meta_items(meta_files, attachments=None):
    """Dataset3.meta_items(): ``meta_files`` = {path relative to the meta tree: bytes} of one
    dataset version (None or empty: no meta tree, no items), ``attachments`` = {name: bytes} of the
    files next to its .table-dataset tree (metadata.xml)."""
    if not meta_files:
        return {}
    attachments = attachments or {}
    out = {}
    for name in META_ITEM_NAMES:
        data = attachments.get(name) if name in ATTACHMENT_META_ITEMS else meta_files.get(name)
        value = meta_item_value(name, data)
        if value:
            out[name] = value
    # crs_definitions: every blob under meta/crs/ (up to 4 levels down, as find_blobs_in_tree goes),
    # identified by its own name minus 4 characters, keyed crs/<identifier>.wkt
    for rel in sorted(p for p in meta_files if p.startswith(CRS_DIR)):
        if rel[len(CRS_DIR):].count("/") > 4:
            continue
        base = rel.rsplit("/", 1)[-1]
        out[f"crs/{base[:-4]}.wkt"] = normalise_wkt(ensure_text(meta_files[rel]))
    return out
