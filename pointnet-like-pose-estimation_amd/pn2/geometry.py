"""Geometry stream: the index work of an SA layer (FPS, ball query) that depends only on an
earlier layer's geometry runs on its own HIP stream, overlapping the earlier layer's grouped MLP.

Dependency rule.  The geometry of layer i+1 reads only layer i's centroids (``new_points``),
which layer i's geometry produced -- it does not need layer i's MLP output.  Every geometry
result is registered with an event recorded right after the launches that produced it.  When
all inputs of a geometry span are registered, the span runs on the geometry stream after
waiting on those events (already passed, or about to), so FPS2 / BQ2 run concurrently with
MLP1; the caller's stream then waits on the span's event before the MLP.  A span with any other
("foreign") input -- the caller's point cloud -- runs on the caller's stream: a cross-stream hop
costs more than it could hide there (measured: ~15-25 us of idle per hop on MI355X).

A registered tensor is recognised by its data pointer while the tensor that owns that memory is
alive and unmodified (same version counter; views share it).  Tensors allocated on the geometry
stream and read on the caller's stream are ``record_stream``-ed there, so the caching allocator
does not recycle them early.

Opt-in with tuning ``geometry_stream`` = 1 (pn2/tuning.py); by default (and inside graph capture) everything stays
on the caller's stream.
"""
import contextlib
import threading
import weakref

import torch

from . import tuning

_streams = {}
_produced = {}  # data_ptr -> (weakref to owning tensor, version, event)


def enabled():
    # opt-in: on MI355X the overlap it buys (FPS2/BQ2 under MLP1, ~40 us) is about what the
    # cross-stream wait and the CU sharing cost (measured 0.8726 vs 0.8713 ms/step, SSG B=32)
    return bool(tuning.get("geometry_stream")) and not torch.cuda.is_current_stream_capturing()


def _stream(device):
    key = torch.device(device).index
    s = _streams.get(key)
    if s is None:
        lo, hi = torch.cuda.Stream.priority_range()
        # FPS is a serial latency chain on the forward's critical path: highest priority
        s = torch.cuda.Stream(device=device, priority=min(lo, hi))
        _streams[key] = s
    return s


def _lookup(t):
    ent = _produced.get(t.data_ptr())
    if ent is None:
        return None
    ref, ver, ev = ent
    owner = ref()
    if owner is None or owner._version != ver:
        return None
    return ev


def _register(t, ev):
    for k in [k for k, (r, _, _) in _produced.items() if r() is None]:
        del _produced[k]
    _produced[t.data_ptr()] = (weakref.ref(t), t._version, ev)


class Span:
    """``with Span(device, inputs) as sp: <geometry launches>; sp.finish(produced, used)``.

    inputs: tensors the geometry launches read.  produced: tensors later geometry may consume
    (registered).  used: geometry outputs the caller's stream reads next."""

    def __init__(self, device, inputs):
        self.main = torch.cuda.current_stream(device)
        evs = [_lookup(t) for t in inputs if t is not None]
        self.side = enabled() and len(evs) > 0 and all(e is not None for e in evs)
        self.stream = self.main
        if self.side:
            self.stream = _stream(device)
            for e in evs:
                self.stream.wait_event(e)
            for t in inputs:
                t.record_stream(self.stream)
        self._ctx = torch.cuda.stream(self.stream)

    def __enter__(self):
        self._ctx.__enter__()
        return self

    def __exit__(self, *exc):
        self._ctx.__exit__(*exc)
        return False

    def finish(self, produced, used):
        if not enabled():
            return
        ev = torch.cuda.Event()
        ev.record(self.stream)
        for t in produced:
            _register(t, ev)
        if self.side:
            self.main.wait_event(ev)
            for t in used:
                t.record_stream(self.main)


# ----------------------------------------------------------------------------- provided FPS
# pn2.pipeline runs a batch's geometry chain (FPS + ball queries of every SA layer) ahead of its
# forward; the SA modules then take the precomputed (centroids, packed centroids, packed
# points, neighbour indices per radius) instead of drawing, sampling and querying.
_tls = threading.local()


@contextlib.contextmanager
def provide(entries):
    """entries: {id(module): (input data_ptr, new_points, ctr_packed, pts_packed, idxs)};
    idxs: the ball query's (indices, distinct-neighbour counts) per radius of the module, or
    None (the module queries)."""
    prev = getattr(_tls, "entries", None)
    _tls.entries = entries
    try:
        yield
    finally:
        _tls.entries = prev


def provided(module):
    """Whether pn2.pipeline provided `module`'s geometry for the current forward."""
    entries = getattr(_tls, "entries", None)
    return bool(entries) and id(module) in entries


# ----------------------------------------------------------------------------- FPS lookahead
# In an eager forward the next SA layer's FPS reads only this layer's centroids: the heads wrap
# sa1 -> sa2 in fps_ahead(sa1, sa2), and sa1's MLP call then runs sa2's FPS as a side job of the
# same launch (pn2_fps_side: extra workgroups of the chain kernel, overlapping the MLP; ~40 us
# off SSG's serial chain).  sa2's start is drawn right after sa1's own, where the reference draws
# it relative to every other draw (nothing draws in between).  Not inside graph capture, with
# geometry provided by pn2.pipeline, or with the geometry stream on.
@contextlib.contextmanager
def fps_ahead(first, nxt):
    prev = getattr(_tls, "pair", None)
    _tls.pair = (first, nxt)
    try:
        yield
    finally:
        _tls.pair = prev
        ahead = getattr(_tls, "ahead", None)
        if ahead:
            ahead.pop(id(nxt), None)  # not taken (an exception on the way): dropped


def ahead_of(module):
    """The module whose FPS `module`'s MLP call may run (fps_ahead), or None."""
    pair = getattr(_tls, "pair", None)
    if pair is None or pair[0] is not module or enabled() or provided(pair[1]):
        return None
    if torch.cuda.is_current_stream_capturing():
        return None
    return pair[1]


def put_ahead(module, pts, newp, cpk, ppk):
    """Register `module`'s FPS results, computed ahead on `pts` (its forward's points)."""
    if not hasattr(_tls, "ahead"):
        _tls.ahead = {}
    _tls.ahead[id(module)] = (pts.data_ptr(), newp, cpk, ppk, None)


def take(module, pts):
    """The provided (pn2.pipeline) or computed-ahead (fps_ahead) FPS results for `module` called
    on `pts`, or None.  An entry whose recorded input differs from `pts` is an error (the
    precomputed sampling -- and the RNG draws behind it -- would not match this call)."""
    ahead = getattr(_tls, "ahead", None)
    if ahead and id(module) in ahead:
        ptr, newp, cpk, ppk, idxs = ahead.pop(id(module))
        if ptr != pts.data_ptr():
            raise RuntimeError("pn2.geometry.fps_ahead: the SA module was called on a different "
                               "point tensor than the centroids its FPS was computed on")
        return newp, cpk, ppk, idxs
    entries = getattr(_tls, "entries", None)
    if not entries or id(module) not in entries:
        return None
    ptr, newp, cpk, ppk, idxs = entries.pop(id(module))
    if ptr != pts.data_ptr():
        raise RuntimeError("pn2.pipeline: the SA module was called on a different point tensor "
                           "than the one its FPS was precomputed for")
    return newp, cpk, ppk, idxs
