"""Extract the anchor / RPN-geometry fields of the reference's 16 config
presets (/root/reference/configs/**/*.json, read as JSON data) into
tests/golden/ref_presets.json.  Only the keys that decide the anchor pyramid
and the RPN head's row count are kept (a derived fixture, not a copy of the
files).  Run from the repo root: python tests/golden/make_ref_presets.py"""
import glob
import json
import os

KEYS = ("MODE", "IMAGE_SIZE", "IMAGE_DEPTH", "IMAGE_CHANNEL_COUNT", "BACKBONE", "BACKBONE_STRIDES",
        "TOP_DOWN_PYRAMID_SIZE", "RPN_ANCHOR_SCALES", "RPN_ANCHOR_RATIOS", "RPN_ANCHOR_STRIDE")
ROOT = "/root/reference/configs"

out = {}
for path in sorted(glob.glob(os.path.join(ROOT, "**", "*.json"), recursive=True)):
    with open(path) as f:
        d = json.load(f)
    out[os.path.relpath(path, ROOT)] = {k: d[k] for k in KEYS if k in d}
with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref_presets.json"), "w") as f:
    json.dump(out, f, indent=1, sort_keys=True)
print(len(out), "presets")
