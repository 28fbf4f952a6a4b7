"""The C ABI library loads (no GPU needed) and exports every symbol include/pn2.h declares;
argument validation happens before any device call, so the error paths run on CPU too."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "pn2.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pn2_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from pn2 import _lib
    L = _lib.load()
    syms = declared_symbols()
    assert len(syms) >= 13
    for s in syms:
        assert hasattr(L, s), s
        assert s in _lib.SIGNATURES, "ctypes binding missing for " + s


def test_abi_constants():
    from pn2 import _lib
    L = _lib.load()
    assert L.pn2_abi_version() == _lib.ABI_VERSION
    assert [L.pn2_packed_stride(c) for c in (3, 4, 10, 11, 16)] == [4, 8, 12, 12, 20]
    assert [L.pn2_layer_cin_pad(c) for c in (3, 8, 131, 259, 323)] == [8, 8, 136, 264, 328]


def test_validation_errors_without_gpu():
    from pn2 import _lib
    L = _lib.load()
    rc = L.pn2_fps_f32(None, 1, 8, 3, 24, 3, 1, None, 4, None, None, None, None, None)
    assert rc == -1 and b"null" in L.pn2_last_error()
    rc = L.pn2_ball_query_f32(1, 1, 2, 8, 4, 3, 0.2, 9, 1, None)
    assert rc == -1 and b"sample_number 9 > N 8" in L.pn2_last_error()
    rc = L.pn2_fps_f32(1, 1, 8, 65, 520, 65, 1, 1, 4, 1, None, None, None, None)
    assert rc == -2 and b"unsupported C" in L.pn2_last_error()


def test_workspace_queries_r03():
    """Host-side size queries of this round's entry points (no device call)."""
    from pn2 import _lib
    L = _lib.load()
    # FPS: register-resident shapes and the streamed kernel with LDS distances need none; past
    # N = 40896 one word per point
    assert L.pn2_fps_workspace_bytes(4, 16384, 3, 512) == 0
    assert L.pn2_fps_workspace_bytes(4, 32768, 3, 512) == 0
    assert L.pn2_fps_workspace_bytes(4, 50000, 3, 256) == 4 * 50000 * 4
    # the LDS holds the 16 double-buffered 8-byte wave slots beside the N words
    assert L.pn2_fps_workspace_bytes(2, 40896, 3, 256) == 0
    assert L.pn2_fps_workspace_bytes(2, 40897, 3, 256) == 2 * 40897 * 4
    assert L.pn2_fps_workspace_bytes(0, 0, 3, 1) == -1
    # the FC tail: y1 and y2, each padded to 4 floats
    assert L.pn2_fc_tail_workspace_bytes(32, 512, 256) == (32 * 512 + 32 * 256) * 4
    assert L.pn2_fc_tail_workspace_bytes(5, 513, 255) == (((5 * 513 + 3) // 4 * 4) + ((5 * 255 + 3) // 4 * 4)) * 4
    assert L.pn2_fc_tail_workspace_bytes(0, 1, 1) == -1


def test_validation_errors_r03_without_gpu():
    from pn2 import _lib
    L = _lib.load()
    # int32 ball query: the same shape checks as the int64 one
    rc = L.pn2_ball_query_i32(1, 1, 2, 8, 4, 3, 0.2, 9, 1, None, None)
    assert rc == -1 and b"sample_number 9 > N 8" in L.pn2_last_error()
    # streamed FPS past N = 40896 without the workspace it needs
    rc = L.pn2_fps_ws_f32(1, 2, 50000, 3, 150000, 3, 1, 1, 16, 1, None, None, None, None, 0, None)
    assert rc == -1 and b"workspace" in L.pn2_last_error()
    rc = L.pn2_fps_f32(1, 2, 50000, 3, 150000, 3, 1, 1, 16, 1, None, None, None, None)
    assert rc == -1 and b"workspace" in L.pn2_last_error()
    # FC tail: a row block's logits must fit its LDS
    rc = L.pn2_fc_tail_f32(1, 1024, 2, 1024, 1, None, 512, 1, None, 256, 1, None, 5000, 1, 1, 5000, None,
                           1 << 20, 1 << 30, None)
    assert rc == -1 and b"N3" in L.pn2_last_error()


def test_tuning_switch_keys():
    """The one tuning switch: the C keys are readable / settable and unknown keys fail."""
    import ctypes
    from pn2 import _lib, tuning
    L = _lib.load()
    keys = L.pn2_tuning_keys().decode().split()
    for k in ("mlp_f32", "compact", "bq_waves", "bq_rowbuf_kb", "fps_threads", "fps_ppt", "dense_lds"):
        assert k in keys
    v = ctypes.c_int64(-1)
    assert L.pn2_tuning_get(b"dense_lds", ctypes.byref(v)) == 0 and v.value == 1
    assert L.pn2_tuning_set(b"no_such_key", 1) != 0
    with tuning.override(fps_threads=512, tail_streams=2):
        assert tuning.kernel("fps_threads") == 512 and tuning.get("tail_streams") == 2
    assert tuning.kernel("fps_threads") == 0 and tuning.get("tail_streams") == 1


def test_pipeline_queue_rule(monkeypatch):
    """The pipeline gives the heads their tail stream(s) only while every stream has a hardware
    queue (GPU_MAX_HW_QUEUES, HIP's default 4)."""
    from pn2 import pipeline
    monkeypatch.delenv("GPU_MAX_HW_QUEUES", raising=False)
    assert pipeline._hw_queues() == 4
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "8")
    assert pipeline._hw_queues() == 8
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "junk")
    assert pipeline._hw_queues() == 4


def _layers(widths, cin):
    from pn2 import _lib
    arr = (_lib.MlpLayer * len(widths))()
    for i, w in enumerate(widths):
        arr[i].wt = arr[i].alpha = arr[i].beta = 16  # dummy non-null (never dereferenced)
        arr[i].cin = cin if i == 0 else widths[i - 1]
        arr[i].cout = w
    return arr


@pytest.mark.parametrize("widths,cin,mode,fused", [
    ([64, 64, 128], 3, 0, True),        # SSG sa1
    ([128, 128, 256], 131, 0, True),    # SSG sa2
    ([32, 32, 64], 3, 1, True),         # MSG sa1 scale 0
    ([64, 96, 128], 3, 1, True),        # MSG sa1 scale 2
    ([128, 128, 256], 323, 1, True),    # MSG sa2 (feature-first, 320 + 3)
    ([256, 512, 1024], 259, 2, False),  # group_all: hidden 512 > 256 -> layer by layer
])
def test_workspace_query(widths, cin, mode, fused):
    from pn2 import _lib
    L = _lib.load()
    s = _lib.SaSrc()
    s.mode = mode
    s.pts = s.ctr = s.idx = s.feat = 16
    s.B, s.N, s.C, s.S, s.K = 2, 1024, 3, 128, 32
    s.D = cin - 3
    if mode == 2:
        s.S, s.K = 1, 1024
    ws = L.pn2_sa_mlp_workspace_bytes(s, _layers(widths, cin), len(widths))
    assert (ws == 0) == fused and ws >= 0


def test_io_library_exports_every_declared_symbol():
    """libpn2io.so (the dataset text reader, host code) against include/pn2io.h."""
    from pn2 import data
    text = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "pn2io.h")).read(), flags=re.S)
    syms = sorted(set(re.findall(r"\b(pn2io_[a-z0-9_]+)\s*\(", text)))
    L = data.load()
    assert len(syms) == 5
    for s in syms:
        assert hasattr(L, s), s
    assert L.pn2io_abi_version() == data.ABI_VERSION
    rc = L.pn2io_read_csv_f64(b"/nonexistent/x.txt", b",", 3, 10, None, None)
    assert rc == -4 and b"bad argument" in L.pn2io_last_error()


def test_tuning_local_is_per_thread():
    """pn2_tuning_local: a thread's own copy of the kernel keys (the pipelines capture under
    their launch profile in it); other threads keep the process-wide values; nesting counts."""
    import threading
    from pn2 import tuning
    base = tuning.kernel("fps_mid")
    seen = {}
    inside = threading.Event()
    release = threading.Event()

    def worker():
        with tuning.pipeline_profile():
            with tuning.local():  # nested enter keeps the copy
                seen["nested"] = tuning.kernel("fps_mid")
            seen["worker"] = tuning.kernel("fps_mid")
            inside.set()
            release.wait(10)
        seen["after"] = tuning.kernel("fps_mid")

    t = threading.Thread(target=worker)
    t.start()
    assert inside.wait(10)
    seen["main"] = tuning.kernel("fps_mid")
    release.set()
    t.join(10)
    assert seen == {"nested": 256, "worker": 256, "main": base, "after": base}
    assert base == 512


def test_pipeline_profile_keeps_explicit_keys():
    """An explicitly set kernel key wins inside the pipelines' launch profile: the
    profile only replaces keys still at their library default."""
    from pn2 import tuning
    assert tuning.kernel_default("fps_mid") == 512 and tuning.kernel_default("dense_lds") == 1
    with tuning.pipeline_profile():
        assert tuning.kernel("fps_mid") == 256 and tuning.kernel("dense_lds") == 0
    with tuning.override(fps_mid=384):
        assert tuning.effective_pipeline_profile() == {"dense_lds": 0, "bq_waves": 0, "dense_pair": 0}
        with tuning.pipeline_profile():
            assert tuning.kernel("fps_mid") == 384 and tuning.kernel("dense_lds") == 0
    with tuning.override(pipe_profile=0):
        assert tuning.effective_pipeline_profile() == {}


def test_tuning_keys_atomic_under_threads():
    """Process-wide kernel keys are atomic words (errors.cpp): concurrent sets and gets from
    several threads always read one of the values written, never a torn one."""
    import threading
    from pn2 import _lib, tuning
    L = _lib.load()
    base = tuning.kernel("dense_minwg")
    vals = {base, (1 << 40) + 7, -(1 << 33)}
    bad = []

    def work(v):
        for _ in range(2000):
            tuning._set_kernel(L, "dense_minwg", v)
            got = tuning.kernel("dense_minwg")
            if got not in vals:
                bad.append(got)
    ts = [threading.Thread(target=work, args=(v,)) for v in vals]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    tuning._set_kernel(L, "dense_minwg", base)
    assert not bad


def test_thread_generator_draws_are_per_thread():
    """pn2.shard.thread_generator: a thread's FPS start draws come from its own generator, so
    concurrent threads draw reproducibly; outside it the CPU default generator (the reference's)."""
    import threading
    import torch
    from pn2 import shard
    g = torch.Generator().manual_seed(5)
    want = torch.randint(0, 1000, (6,), generator=g)
    want_into = torch.randint(0, 1000, (6,), generator=g)
    got = {}

    def work(k):
        with shard.thread_generator(torch.Generator().manual_seed(5)):
            got[k] = shard.draw_start(6, 1000, pin=False)
            dst = torch.empty(6, dtype=torch.long)
            shard.draw_start_into(dst, 1000)
            got[k, "into"] = dst
    torch.manual_seed(1)
    ref_default = torch.randint(0, 1000, (6,))
    ts = [threading.Thread(target=work, args=(k,)) for k in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for k in range(4):
        assert torch.equal(got[k], want) and torch.equal(got[k, "into"], want_into)
    torch.manual_seed(1)
    assert torch.equal(shard.draw_start(6, 1000, pin=False), ref_default)


def test_error_slot_api_exported():
    """ABI 14: per-thread device error slots and the tuning defaults are exported."""
    from pn2 import _lib
    L = _lib.load()
    for name in ("pn2_error_slot_set", "pn2_error_slot_take", "pn2_device_errors",
                 "pn2_tuning_default"):
        assert hasattr(L, name)
    import ctypes
    v = ctypes.c_int64(0)
    assert L.pn2_tuning_default(b"no_such_key", ctypes.byref(v)) != 0


def test_asm_read_checker_flags_violations():
    """tools/check_asm_reads.py (run by the build on sa_chain.hip's device assembly) flags a
    pending inline-asm LDS read whose registers are touched, or carried across a branch to a
    target that does not wait, before its s_waitcnt; and accepts the covered forms."""
    import importlib.util
    import io
    spec = importlib.util.spec_from_file_location("car", os.path.join(ROOT, "tools", "check_asm_reads.py"))
    car = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(car)
    head = "_ZN3pn215sa_chain_kernelILi1EEEvv:\n"
    rd = ";;#ASMSTART\nds_read_b128 v[4:7], v1\n;;#ASMEND\n"
    tail = ".Lfunc_end0:\n"
    ok = head + rd + "s_waitcnt lgkmcnt(0)\nv_mov_b32 v9, v5\n" + tail
    touch = head + rd + "v_mov_b32 v9, v5\ns_waitcnt lgkmcnt(0)\n" + tail
    younger = head + "ds_read_b32 v20, v2\n" + rd + "s_waitcnt lgkmcnt(1)\nv_mov_b32 v9, v6\n" + tail
    covered = head + rd + "ds_read_b32 v20, v2\ns_waitcnt lgkmcnt(0)\nv_mov_b32 v9, v6\n" + tail
    br_bad = head + rd + "s_cbranch_scc1 .LBB0_2\ns_waitcnt lgkmcnt(0)\n.LBB0_2:\nv_mov_b32 v9, v1\n" + tail
    br_ok = head + rd + "s_cbranch_scc1 .LBB0_2\ns_waitcnt lgkmcnt(0)\n.LBB0_2:\ns_waitcnt lgkmcnt(0)\n" + tail
    sink = io.StringIO()
    assert car.check(ok, sink) == 0
    assert car.check(touch, sink) == 1
    assert car.check(younger, sink) == 1
    assert car.check(covered, sink) == 0
    assert car.check(br_bad, sink) == 1
    assert car.check(br_ok, sink) == 0
