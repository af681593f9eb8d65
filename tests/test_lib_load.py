"""m3d._lib.load(): the library file switch used by A/B builds (CPU only, no
compute calls)."""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_lib_file_switch_selects_the_library(tmp_path):
    """M3D_LIB_FILE (A/B builds, `make ab`) names another build in m3d/: a name
    that does not exist raises at load, never falls back."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import m3d._lib as L\n"
            "try:\n    L.load()\nexcept L.M3DError as e:\n    print('raised', 'libm3d_nonexistent.so' in str(e))\n"
            % os.path.join(ROOT, "3d-mask-r-cnn_amd"))
    env = dict(os.environ, M3D_LIB_FILE="libm3d_nonexistent.so")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert out.stdout.strip() == "raised True", out.stdout + out.stderr
