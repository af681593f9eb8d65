"""m3d_stream_fork (the weight-gradient stream's fork / join, m3d.nn._fork):
work enqueued on the destination after the fork sees everything the source
stream wrote before it, for every event kind (the caller-owned events of
m3d_fork_event_create, ABI 3); a bad mode / NULL event is rejected."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_stream_fork_orders_work(cuda, mode):
    import m3d._lib as lib
    from m3d.nn import fork_event
    L = lib.load()
    a, b = torch.cuda.Stream(cuda), torch.cuda.Stream(cuda)
    n = 1 << 24
    for it in range(4):
        with torch.cuda.stream(a):
            x = torch.empty(n, device=cuda)
            x.fill_(float(it + 1))
            for _ in range(8):                         # keep stream a busy past the fork
                x.mul_(1.0000001)
            y = x * 2.0
        lib.check(L.m3d_stream_fork(a.cuda_stream, b.cuda_stream, fork_event(cuda.index or 0, mode)), "stream_fork")
        with torch.cuda.stream(b):
            s = y.sum()
        y.record_stream(b)
        lib.check(L.m3d_stream_fork(b.cuda_stream, torch.cuda.current_stream(cuda).cuda_stream,
                                    fork_event(cuda.index or 0, mode)), "stream_fork")
        want = 2.0 * (it + 1) * (1.0000001 ** 8) * n
        assert abs(float(s) - want) <= 1e-5 * want


def test_stream_fork_bad_mode(cuda):
    import ctypes

    import m3d._lib as lib
    s = torch.cuda.current_stream(cuda).cuda_stream
    ev = ctypes.c_void_p()
    with pytest.raises(ValueError):
        lib.check(lib.load().m3d_fork_event_create(3, ctypes.byref(ev)), "fork_event_create")
    with pytest.raises(ValueError):
        lib.check(lib.load().m3d_stream_fork(s, s, None), "stream_fork")
    lib.check(lib.load().m3d_fork_event_create(2, ctypes.byref(ev)), "fork_event_create")
    lib.check(lib.load().m3d_stream_fork(s, s, ev.value), "stream_fork")
    torch.cuda.synchronize()
    lib.check(lib.load().m3d_fork_event_destroy(ev.value), "fork_event_destroy")


def test_stream_handle_is_torch_current_stream(cuda):
    """m3d._lib.stream() (the raw-handle fast path) names the stream torch
    considers current, on the default stream and inside a side-stream context."""
    from m3d import _lib
    assert _lib.stream() == torch.cuda.current_stream().cuda_stream
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        assert _lib.stream() == side.cuda_stream == torch.cuda.current_stream().cuda_stream
    assert _lib.stream() == torch.cuda.current_stream().cuda_stream


def test_fork_mode2_recycled_buffers(cuda):
    """The weight-gradient fork's default event kind (mode 2: no system-scope
    fence) with buffers the caching allocator recycles between the streams: a
    block written on one stream, handed to the other by the fork, freed and
    reused there, always reads back what its last writer stored (the
    device-scope release of each kernel's end carries it across XCDs)."""
    import m3d._lib as lib
    from m3d.nn import fork_event
    L = lib.load()
    side, main = torch.cuda.Stream(cuda), torch.cuda.current_stream(cuda)
    n = 1 << 20
    for it in range(64):
        with torch.cuda.stream(side):
            x = torch.full((n,), float(it), device=cuda)
            x.add_(0.5)
        lib.check(L.m3d_stream_fork(side.cuda_stream, main.cuda_stream, fork_event(cuda.index or 0, 2)), "fork")
        s = x.sum()                                   # main reads the side stream's block
        x.record_stream(main)
        del x                                         # the block returns to side's pool after main's use
        lib.check(L.m3d_stream_fork(main.cuda_stream, side.cuda_stream, fork_event(cuda.index or 0, 2)), "fork")
        with torch.cuda.stream(side):
            y = torch.full((n,), -1.0, device=cuda)   # likely the recycled block, rewritten
            t = y.sum()
        lib.check(L.m3d_stream_fork(side.cuda_stream, main.cuda_stream, fork_event(cuda.index or 0, 2)), "fork")
        assert float(s) == (it + 0.5) * n
        assert float(t) == -float(n)
        del y
