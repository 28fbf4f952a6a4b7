"""Concurrent host threads on one device -- the reference's mutilthreading/predict_test.py:44-63
pattern (four heads, four Python threads, one GPU) -- through the drop-in (the C ABI
must be re-entrant, with no global mutable state on the launch path).

  * four threads, each running a different head (cls_ssg, rotation_ssg, translation_ssg,
    sign_ssg) on its own torch stream, concurrently, 20 forwards each: every output bit-equal
    to the same head run serially with the same start draws (each thread draws from its own
    generator, pn2.shard.thread_generator);
  * a fifth thread launches an out-of-range index_points on its own stream every iteration: its
    check_device_errors() raises IndexError every time, and no other thread's ever does (the
    device error slots are per thread, include/pn2.h pn2_error_slot_set);
  * kernel tuning keys set on one thread while the others launch (atomic words).
"""
import threading
import time

import pytest
import torch

import cases

pytestmark = pytest.mark.gpu
DEV = "cuda"
ITERS = 20
B, N = 4, 1024

# name -> (head, cloud kind, weight seed, generator seed)
HEADS = {
    "cls_ssg": ("pointnet2_cls_ssg", "uniform3", 300, 400),
    "rotation_ssg": ("rotation_ssg", "onehot10", 301, 401),
    "translation_ssg": ("translation_ssg", "onehot10", 302, 402),
    "sign_ssg": ("sign_ssg", "onehot10", 303, 403),
}


def _setup():
    from pn2 import heads as H
    out = {}
    for name, (head, kind, wseed, gseed) in HEADS.items():
        model = cases.build_head(H.HEADS[head], wseed).to(DEV).eval()
        x = cases.cloud(kind, B, N, wseed + 7).permute(0, 2, 1).contiguous().to(DEV)
        args = [x]
        if head.startswith("translation"):
            args.append(torch.randn(B, 3, generator=torch.Generator().manual_seed(wseed)).to(DEV))
        out[name] = (model, args, gseed)
    return out


def _flat(out):
    ts = out if isinstance(out, (tuple, list)) else (out,)
    return [t.detach().clone() for t in ts]


def _run_head(model, args, gseed, iters, stream, barrier=None, after=None):
    from pn2 import shard
    res = []
    g = torch.Generator().manual_seed(gseed)
    with torch.no_grad(), torch.cuda.stream(stream), shard.thread_generator(g):
        if barrier is not None:
            barrier.wait()
        for _ in range(iters):
            res.append(_flat(model(*args)))
            if after is not None:
                after()
    stream.synchronize()
    return [[t.cpu() for t in r] for r in res]


def _bad_index_loop(iters, stream, barrier, log):
    import pn2
    from pn2 import ops
    with torch.cuda.stream(stream):
        pts = torch.rand(2, 64, 3, device=DEV)
        idx = torch.full((2, 5), 64, dtype=torch.int64, device=DEV)  # outside [-64, 64)
        barrier.wait()
        for _ in range(iters):
            out = ops.index_points_direct(pts, idx)
            try:
                pn2.check_device_errors()
            except IndexError:
                log.append("raised")
            else:
                log.append("missed")
            assert torch.isnan(out).all()


def _threads(targets):
    errs = []

    def wrap(fn):
        def run():
            try:
                fn()
            except BaseException as e:  # re-raised on the main thread
                errs.append(e)
        return run
    ts = [threading.Thread(target=wrap(f)) for f in targets]
    for t in ts:
        t.start()
    for t in ts:
        t.join(300)
        assert not t.is_alive(), "thread did not finish"
    if errs:
        raise errs[0]


def test_four_heads_on_four_threads_match_serial():
    import pn2
    setup = _setup()
    pn2.check_device_errors()  # nothing pending
    serial = {name: _run_head(m, a, gs, ITERS, torch.cuda.Stream()) for name, (m, a, gs) in setup.items()}

    barrier = threading.Barrier(len(setup) + 1)
    got, bad_log = {}, []

    def head_thread(name):
        m, a, gs = setup[name]
        # every forward's own bits: none (the bad-index thread's IndexErrors are its own)
        got[name] = _run_head(m, a, gs, ITERS, torch.cuda.Stream(), barrier,
                              after=pn2.check_device_errors)

    _threads([lambda n=n: head_thread(n) for n in setup] +
             [lambda: _bad_index_loop(ITERS, torch.cuda.Stream(), barrier, bad_log)])
    assert bad_log == ["raised"] * ITERS
    for name in setup:
        assert len(got[name]) == ITERS
        for i, (g, s) in enumerate(zip(got[name], serial[name])):
            for a, b in zip(g, s):
                assert torch.equal(a, b), "%s forward %d differs from the serial run" % (name, i)
    pn2.check_device_errors()  # the main thread raised nothing either


def test_device_errors_are_per_thread():
    """A bit raised on one thread is invisible to, and not cleared by, another thread's check."""
    import pn2
    from pn2 import ops
    pn2.check_device_errors()
    pts = torch.rand(1, 16, 3, device=DEV)
    bad = torch.full((1, 2), 99, dtype=torch.int64, device=DEV)
    raised = threading.Event()
    checked = threading.Event()
    log = {}

    def raiser():
        ops.index_points_direct(pts, bad)
        torch.cuda.synchronize()
        raised.set()
        assert checked.wait(60)
        try:
            pn2.check_device_errors()
        except IndexError:
            log["raiser"] = "raised"

    def checker():
        assert raised.wait(60)
        pn2.check_device_errors()  # must not raise, nor take the other thread's bit
        log["checker"] = "clean"
        checked.set()

    _threads([raiser, checker])
    assert log == {"raiser": "raised", "checker": "clean"}


def test_tuning_set_while_other_threads_launch():
    """Process-wide kernel keys are atomic words: flipping a launch choice on one thread while
    other threads run forwards neither crashes nor changes results (both forms are exact)."""
    from pn2 import _lib, tuning
    from pn2 import heads as H
    head, kind, wseed, gs = HEADS["cls_ssg"]
    models = [cases.build_head(H.HEADS[head], wseed).to(DEV).eval() for _ in range(3)]
    a = [cases.cloud(kind, B, N, wseed + 7).permute(0, 2, 1).contiguous().to(DEV)]
    ref = _run_head(models[0], a, gs, 4, torch.cuda.Stream())
    stop = threading.Event()
    got = {}
    L = _lib.load()

    def flipper():
        v = tuning.kernel("bq_waves")
        i = 0
        while not stop.is_set():
            tuning._set_kernel(L, "bq_waves", 8 if i % 2 else 16)
            i += 1
            time.sleep(0.0002)
        tuning._set_kernel(L, "bq_waves", v)

    def runner(k):
        got[k] = _run_head(models[k], a, gs, 4, torch.cuda.Stream())

    ft = threading.Thread(target=flipper)
    ft.start()
    try:
        _threads([lambda k=k: runner(k) for k in range(3)])
    finally:
        stop.set()
        ft.join(30)
    for k in range(3):
        for g, s in zip(got[k], ref):
            for x, y in zip(g, s):
                assert torch.equal(x, y)
