"""bench.py with module constants of the host path set first (A/B of the
Python-side switches without environment variables):

    python scripts/bench_ab.py nn.X3_BN_FUSE=0,backbone.BN_AFFINE_BATCHED=0 -- --steps 20 --no-extras
"""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]


def main():
    spec, rest = sys.argv[1], sys.argv[sys.argv.index("--") + 1:]
    for item in filter(None, spec.split(",")):
        key, val = item.split("=")
        mod, attr = key.rsplit(".", 1)
        m = importlib.import_module("m3d." + mod)
        old = getattr(m, attr)
        setattr(m, attr, type(old)(int(val)) if isinstance(old, (bool, int)) else type(old)(val))
    sys.argv = ["bench.py"] + rest
    import bench
    bench.main()


if __name__ == "__main__":
    main()
