"""Extract the reference's own hex-WKB golden values (tests/test_diff.py, `kart diff -o json`
of HEAD^...HEAD on the points and polygons repos) into tests/golden/hexwkb.json.

Reads the reference test file as text (ast.literal_eval of the expected-output dict literals;
nothing is imported or executed).  Run here only: python tests/golden/gen_hexwkb.py
"""
import ast
import json
import os

SRC = "/root/reference/tests/test_diff.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hexwkb.json")
DATASETS = {"nz_pa_points_topo_150k": ("repo_points", "fid"), "nz_waca_adjustments": ("repo_polygons", "id")}


def main():
    tree = ast.parse(open(SRC).read())
    recs = set()
    for node in ast.walk(tree):
        if not isinstance(node, ast.Dict):
            continue
        keys = [k.value for k in node.keys if isinstance(k, ast.Constant)]
        if "kart.diff/v1+hexwkb" not in keys:
            continue
        try:
            d = ast.literal_eval(node)
        except ValueError:
            continue
        for ds, body in d["kart.diff/v1+hexwkb"].items():
            if ds not in DATASETS or not isinstance(body, dict):
                continue
            fixture, pkcol = DATASETS[ds]
            for delta in body.get("feature", []):
                for sign, side in (("-", "head1"), ("+", "head")):
                    if sign in delta and "geom" in delta[sign]:
                        recs.add((fixture, side, int(delta[sign][pkcol]), delta[sign]["geom"]))
    out = [{"fixture": f, "side": s, "pk": p, "hex": h} for f, s, p, h in sorted(recs)]
    with open(OUT, "w") as fh:
        json.dump(out, fh, indent=1)
    print(f"{len(out)} hex-WKB golden values -> {OUT}")


if __name__ == "__main__":
    main()
