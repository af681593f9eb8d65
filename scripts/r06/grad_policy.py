"""Runs pytest with nn.WINO_DGRAD_Y4 set: grad_policy.py POLICY pytest-args..."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
import pytest  # noqa: E402

from m3d import nn as mnn  # noqa: E402

mnn.WINO_DGRAD_Y4 = sys.argv[1]
sys.exit(pytest.main(sys.argv[2:]))
