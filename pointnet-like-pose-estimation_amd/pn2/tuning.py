"""Tuning of the launch choices -- for A/B experiments and tests, not for users.

The product path reads one environment variable, once, at import:

    PN2_TUNING="key=value,key=value,..."

Keys are the library's kernel-selection parameters (include/pn2.h ``pn2_tuning_set``:
``mlp_f32``, ``chain_prepass``, ``dense_pair``, ``compact``, ``compact_pool``, ``compact_stages``,
``bq_waves``, ``bq_rowbuf_kb``, ``fps_threads``, ``fps_ppt``, ``fps_mid``, ``dense_maxntc``,
``dense_minwg``, ``dense_wide_minwg``, ``dense_lds``, ``dense_lds_stages``, ``dense_lds_xcd2d``,
``dense_lds_tile``; csrc/pn2_internal.h documents each) and these host-side ones:

    tail_prio        1: the pipeline's tail stream at high priority
    heads_on_compute 1: the pipeline's heads on the compute streams, no tail stream
    pipe_split_last  1: the pipeline's compute/tail split after the last SA layer
    drain_heads      how many final batches of a pipelined run take their heads on their own
                     compute streams (default 2)
    geometry_stream  1: the eager forward runs layer i+1's FPS + ball query on a side stream
    fc_tail          0: the heads' FC tail as one row-kernel launch per layer + torch's
                     log_softmax / argmax, instead of pn2_fc_tail_f32's fused fc3 + log_softmax
    tail_streams     2: the pipeline's heads alternate between two tail streams (needs the
                     hardware queues: GPU_MAX_HW_QUEUES >= the pipeline's streams)
    force_gather     1: shard.all_gather_rows runs its collective in a 1-rank group too (the
                     bench's --force-rccl measurement of the collective's cost on one GPU)
    geometry_bq      1: the pipeline's geometry stream runs the ball queries after the FPS;
                     0: only the FPS, each batch's forward (compute stream) queries
    pipe_fuse        1: GraphedPipeline runs one forward (sa + head graphs) per geometry group,
                     its batches side by side; 0: one forward per batch
    bq_multi         1: an MSG layer's ball queries in one launch over its radii
                     (pn2_ball_query_multi_i32); 0: one launch per radius
    pipe_profile     1: the pipelines (pn2.pipeline) whose launches carry >= 64 clouds
                     (fused groups, or B >= 64) capture and run their kernels under
                     PIPELINE_PROFILE -- the launch choices measured best beside each other's
                     kernels, where the kernel defaults are the ones measured best alone (the
                     eager forward, GraphedForward); 0: the defaults everywhere; 2: every
                     pipeline (A/B)

Unknown keys are an error.  ``override(**kw)`` changes keys for the duration of a ``with``
block (tests); process-wide kernel keys are atomic words in the library, so a change on one
thread while another launches is safe.  ``pipeline_profile()`` applies PIPELINE_PROFILE only
to keys still at their library default: an explicit setting wins inside the pipelines too.
Every default is the measured best.
"""
import contextlib
import os

HOST_DEFAULTS = {
    "pipe_profile": 1,
    "tail_prio": 0,
    "heads_on_compute": 0,
    "pipe_split_last": 0,
    "drain_heads": 2,
    "geometry_stream": 0,
    "fc_tail": 1,
    "force_gather": 0,
    "tail_streams": 1,
    "geometry_bq": 1,
    "pipe_fuse": 1,
    "bq_multi": 1,
}


def _parse(text):
    out = {}
    for item in filter(None, (t.strip() for t in text.split(","))):
        if "=" not in item:
            raise ValueError("PN2_TUNING: expected key=value, got %r" % item)
        k, v = (s.strip() for s in item.split("=", 1))
        out[k] = int(v)
    return out


_ENV = _parse(os.environ.get("PN2_TUNING", ""))
_host = dict(HOST_DEFAULTS)
_host.update({k: v for k, v in _ENV.items() if k in HOST_DEFAULTS})


# Kernel keys the pipelines set while they capture / run: the FPS block of 4
# waves x 4 points, the register-staged dense kernel, 8-wave ball-query workgroups (for
# clouds below 2048 points) and group_all's first two layers one launch each (the fused pair
# streams both layers' weights per 32-row block: at a fused group's 16384 rows that L2 -> CU
# stream costs more than the launch it saves, SSG K=100 192.2k with it vs 195.3k) -- each
# faster alone in the other form, slower beside the chains.
PIPELINE_PROFILE = {"fps_mid": 256, "dense_lds": 0, "bq_waves": 0, "dense_pair": 0}


@contextlib.contextmanager
def local():
    """Context: this host thread's own copy of the kernel keys (pn2_tuning_local); changes
    inside it do not reach other threads and end with it."""
    from . import _lib
    L = _lib.load()
    _lib.check(L.pn2_tuning_local(1), "pn2_tuning_local")
    try:
        yield
    finally:
        _lib.check(L.pn2_tuning_local(0), "pn2_tuning_local")


_DEFAULTS = {}


def kernel_default(key):
    """A kernel-selection parameter's library default (pn2_tuning_default)."""
    if key not in _DEFAULTS:
        import ctypes
        from . import _lib
        v = ctypes.c_int64(0)
        _lib.check(_lib.load().pn2_tuning_default(key.encode(), ctypes.byref(v)), "pn2_tuning_default")
        _DEFAULTS[key] = v.value
    return _DEFAULTS[key]


def effective_pipeline_profile():
    """The PIPELINE_PROFILE entries a pipeline applies now: only keys that still hold their
    library default -- a key set by PN2_TUNING or override() keeps that value in the pipelines
    too (an A/B of e.g. dense_lds=1 measures the pipelines as well).  {} with pipe_profile 0."""
    if not _host["pipe_profile"]:
        return {}
    return {k: v for k, v in PIPELINE_PROFILE.items() if kernel(k) == kernel_default(k)}


@contextlib.contextmanager
def pipeline_profile():
    """Context: the effective PIPELINE_PROFILE (above) applied on this thread's own copy of
    the keys -- a forward on another host thread meanwhile keeps the defaults."""
    prof = effective_pipeline_profile()
    if not prof:
        yield
        return
    with local(), override(**prof):
        yield


def get(key):
    """A host-side key's value (kernel keys: ``kernel(key)``)."""
    return _host[key]


def kernel(key):
    """A kernel-selection parameter's current value in the loaded library."""
    import ctypes
    from . import _lib
    v = ctypes.c_int64(0)
    _lib.check(_lib.load().pn2_tuning_get(key.encode(), ctypes.byref(v)), "pn2_tuning_get")
    return v.value


def _set_kernel(L, key, value):
    if L.pn2_tuning_set(key.encode(), int(value)) != 0:
        raise ValueError("pn2 tuning: %s" % L.pn2_last_error().decode(errors="replace"))


def apply_env(L):
    """Apply PN2_TUNING's kernel keys to the just-loaded library L (called by _lib.load)."""
    for k, v in _ENV.items():
        if k not in HOST_DEFAULTS:
            _set_kernel(L, k, v)


@contextlib.contextmanager
def override(**kw):
    """Change tuning keys (host-side or kernel) within a ``with`` block, then restore them."""
    from . import _lib
    L = _lib.load()
    saved = []
    try:
        for k, v in kw.items():
            if k in HOST_DEFAULTS:
                saved.append((k, _host[k], True))
                _host[k] = v
            else:
                saved.append((k, kernel(k), False))
                _set_kernel(L, k, v)
        yield
    finally:
        for k, v, host in reversed(saved):
            if host:
                _host[k] = v
            else:
                _set_kernel(L, k, v)
