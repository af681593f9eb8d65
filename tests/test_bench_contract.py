"""bench.py's measurement labels (CPU only): the headline `roofline` prices
the step's dominant kernel, i.e. the kernel on line 1 of the committed rocprof
table of the same tree (profiles/dominant_kernel_table.txt, a copy of the
latest `*_bench_kernels*.txt` summary); VERDICT r4 weak 8."""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_headline_roofline_is_the_dominant_kernel():
    sys.path.insert(0, ROOT)
    import bench
    first = open(os.path.join(ROOT, "profiles", "dominant_kernel_table.txt")).readline()
    m = re.search(r"m3d::(\w+)", first)
    assert m, first
    assert m.group(1) == bench.DOMINANT_KERNEL, (first, bench.DOMINANT_KERNEL)


def test_every_leg_resets_the_peak_memory_counter():
    """peak_mem_gb of a leg is that leg's own peak (reset_peak_memory_stats
    before it), not the process's."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    for fn in ("def depth_slab_leg", "def mrcnn_inference_leg"):
        body = src[src.index(fn):]
        body = body[:body.index("\ndef ", 1)]
        assert "reset_peak_memory_stats" in body, fn
