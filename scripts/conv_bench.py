"""Per-layer TFLOP/s of the conv kernels (fwd / bwd-data / bwd-weight) at the
128^3 RPN shapes.  Diagnostic for kernel tuning; times with HIP events on the
current stream."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
import torch  # noqa: E402

from m3d import _lib  # noqa: E402
from m3d.nn import conv_geom  # noqa: E402

S = int(os.environ.get("S", "128"))
q = S // 4
SHAPES = [  # name, (H,W,D), Cin, Cout, k, stride, padding
    ("stem7", (S, S, S), 1, 64, 7, (2, 2, 1), 3),
    ("s2_1x1_64_256", (q, q, S), 64, 256, 1, (1, 1, 1), "valid"),
    ("s2_1x1_256_64", (q, q, S), 256, 64, 1, (1, 1, 1), "valid"),
    ("s2_3x3_64", (q, q, S), 64, 64, 3, (1, 1, 1), "same"),
    ("s3_1x1s2_256_128", (q, q, S), 256, 128, 1, (2, 2, 1), "valid"),
    ("s3_3x3_128", (q // 2, q // 2, S), 128, 128, 3, (1, 1, 1), "same"),
    ("s3_1x1_128_512", (q // 2, q // 2, S), 128, 512, 1, (1, 1, 1), "valid"),
    ("s4_3x3_256", (q // 4, q // 4, S), 256, 256, 3, (1, 1, 1), "same"),
    ("s4_1x1_1024_256", (q // 4, q // 4, S), 1024, 256, 1, (1, 1, 1), "valid"),
    ("s5_3x3_512", (q // 8, q // 8, S), 512, 512, 3, (1, 1, 1), "same"),
    ("s5_1x1_512_2048", (q // 8, q // 8, S), 512, 2048, 1, (1, 1, 1), "valid"),
    ("fpn_3x3_P2", (q, q, S), 256, 256, 3, (1, 1, 1), "same"),
    ("rpn_3x3_P2", (q, q, S), 256, 512, 3, (1, 1, 1), "same"),
    ("rpn_1x1_P2", (q, q, S), 512, 256, 1, (1, 1, 1), "valid"),
]


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps / 1e3


def main():
    L = _lib.load()
    dev = torch.device("cuda")
    st = _lib.stream
    tot = {"fwd": [0, 0], "dgrad": [0, 0], "wgrad": [0, 0]}
    print(f"{'layer':22s} {'fwd TF/s':>9s} {'dgrad':>9s} {'wgrad':>9s}   (ms fwd/dgrad/wgrad)")
    for name, sp, cin, cout, k, stride, pad in SHAPES:
        g = conv_geom(sp, (k, k, k), stride, pad)
        x = torch.randn((1, *sp, cin), device=dev)
        w = torch.randn((k, k, k, cin, cout), device=dev) * 0.01
        b = torch.zeros(cout, device=dev)
        y = torch.empty((1, *g.out, cout), device=dev)
        dz = torch.randn_like(y)
        dx = torch.zeros_like(x)
        dw = torch.zeros_like(w)
        M = g.out[0] * g.out[1] * g.out[2]
        fl = 2.0 * M * k ** 3 * cin * cout
        H, W, D = sp
        OH, OW, OD = g.out
        f = lambda: _lib.check(L.m3d_conv3d_fwd(x.data_ptr(), 1, H, W, D, cin, w.data_ptr(), k, k, k, cout, OH, OW, OD,  # noqa: E731
                                                *stride, *g.pad, b.data_ptr(), None, None, None, 0, 1, None,
                                                y.data_ptr(), cout, None, 0, 0, st()))
        tf = timeit(f)
        td = float("nan")
        if cin % 4 == 0 and (k == 1 or stride == (1, 1, 1)):
            d = lambda: _lib.check(L.m3d_conv3d_bwd_data(dz.data_ptr(), w.data_ptr(), 1, H, W, D, cin, k, k, k, cout,  # noqa: E731
                                                         OH, OW, OD, *stride, *g.pad, dx.data_ptr(), 0, st()))
            td = timeit(d)
        wg = lambda: _lib.check(L.m3d_conv3d_bwd_weight(x.data_ptr(), dz.data_ptr(), 1, H, W, D, cin, k, k, k, cout,  # noqa: E731
                                                        OH, OW, OD, *stride, *g.pad, dw.data_ptr(), st()))
        tw = timeit(wg)
        if k == 3 and stride == (1, 1, 1) and cin % 32 == 0:
            nb = int(L.m3d_conv3d_wino_workspace_bytes(1, H, W, D, D, cin, cout))
            ws = torch.empty(nb // 4 + 1, device=dev)
            fw = lambda: _lib.check(L.m3d_conv3d_fwd_wino(x.data_ptr(), 1, H, W, D, cin, w.data_ptr(), cout, D, 1,  # noqa: E731
                                                          b.data_ptr(), None, None, None, 1, None, y.data_ptr(),
                                                          ws.data_ptr(), nb, st()))
            dw_ = lambda: _lib.check(L.m3d_conv3d_bwd_data_wino(dz.data_ptr(), w.data_ptr(), 1, H, W, D, cin, cout, D, 1,  # noqa: E731
                                                                dx.data_ptr(), 0, ws.data_ptr(), nb, st()))
            ww = lambda: _lib.check(L.m3d_conv3d_bwd_weight_wino(x.data_ptr(), dz.data_ptr(), 1, H, W, D, cin, cout, D, 1,  # noqa: E731
                                                                 dw.data_ptr(), ws.data_ptr(), nb, st()))
            a, b2, c = timeit(fw), timeit(dw_), timeit(ww)
            print(f"{'  +wino ' + name:22s} {fl / a / 1e12:9.1f} {fl / b2 / 1e12:9.1f} {fl / c / 1e12:9.1f}   "
                  f"({a * 1e3:.3f} / {b2 * 1e3:.3f} / {c * 1e3:.3f})  [direct-equivalent TF/s]", flush=True)
            tf, td, tw = min(tf, a), min(td, b2), min(tw, c)
        for key, t in (("fwd", tf), ("dgrad", td), ("wgrad", tw)):
            if t == t:
                tot[key][0] += fl
                tot[key][1] += t
        print(f"{name:22s} {fl / tf / 1e12:9.1f} {fl / td / 1e12:9.1f} {fl / tw / 1e12:9.1f}   "
              f"({tf * 1e3:.3f} / {td * 1e3:.3f} / {tw * 1e3:.3f})", flush=True)
    for key, (fl, t) in tot.items():
        print(f"TOTAL {key}: {fl / t / 1e12:.1f} TF/s over {t * 1e3:.2f} ms")


if __name__ == "__main__":
    main()
