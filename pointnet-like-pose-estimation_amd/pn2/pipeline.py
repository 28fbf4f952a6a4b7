"""Pipelined eval forward over a stream of batches, with the GPU partitioned by CUs.

Every SA layer's farthest point sampling depends only on the point coordinates (sa1 samples the
input cloud, sa2 the centroids sa1 chose, ...), never on an MLP output, so a batch's whole FPS
chain can run before its forward.  ``PipelinedForward`` runs the FPS chain of batch i+1 while
the ball queries, MLPs and head of batch i run, on two HIP streams that own disjoint CU sets
(hipExtStreamCreateWithCUMask through pn2_stream_create_cu_masked): FPS is a serial,
latency-bound loop of one workgroup per cloud, so it gets a few dedicated CUs instead of
time-sharing CUs with MFMA work (which slows its loop ~2.7x, measured), and the MFMA kernels
keep the rest of the chip.

Results and RNG.  Every batch computes what ``model(x)`` computes: the SA layers run the same
kernels and produce the same bits (test_pipelined_forward_matches_eager); the head's own
``nn.Linear`` layers go through torch's BLAS, which may choose a different GEMM kernel on the
CU-restricted stream (last-ulp differences in logits).  The reference draws one ``torch.randint(0, N, (B,))`` per SA layer from the CPU
generator (pointnet2_utils.py:59); here batch i's draws (all its layers, in layer order) are
taken before batch i+1's -- the order a sequence of eager forwards takes them -- so
``run(batches)`` matches ``[model(x) for x in batches]`` and leaves the generator in the same
state.  ``shard.batch_shard`` slicing applies as in eager.

Scope: eval mode (no autograd), heads whose SA layers are called in registration order on the
previous layer's centroids (every reference head).  Inputs must be ready on the caller's
stream when ``run`` is called.
"""
import atexit
import ctypes

import torch

from . import _lib
from . import geometry
from . import ops
from . import shard
from .pointnet2_utils import PointNetSetAbstraction, PointNetSetAbstractionMsg

_partitions = {}  # (device, geometry CUs) -> (geometry stream, compute stream, raw handles)


@atexit.register
def _destroy_partitions():
    """Release the CU-masked streams before the HIP runtime tears down (left to process exit,
    their destruction raced the runtime's own teardown under rocprofv3)."""
    for key, (_, _, raw) in list(_partitions.items()):
        try:
            torch.cuda.synchronize(key[0])
        except Exception:
            pass
        for h in raw:
            _lib.load().pn2_stream_destroy(h)
    _partitions.clear()


def _cu_count(device):
    n = ctypes.c_int(0)
    _lib.check(_lib.load().pn2_device_cu_count(device, ctypes.byref(n)), "pn2_device_cu_count")
    return n.value


def _masked_stream(device, cus, ncu):
    words = (ncu + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for c in cus:
        mask[c // 32] |= 1 << (c % 32)
    ptr = ctypes.c_void_p()
    _lib.check(_lib.load().pn2_stream_create_cu_masked(device, mask, words, ctypes.byref(ptr)),
               "pn2_stream_create_cu_masked")
    return torch.cuda.ExternalStream(ptr.value, device=torch.device("cuda", device)), ptr.value


def partition(device, geometry_cus):
    """(geometry stream, compute stream) on `device`: `geometry_cus` CUs spread evenly over the
    chip for the FPS chain, all the others for everything else.  Cached per (device, count)."""
    key = (device, geometry_cus)
    if key not in _partitions:
        ncu = _cu_count(device)
        g = max(1, min(int(geometry_cus), ncu - 1))
        stride = ncu / g
        geo = sorted({int(i * stride) for i in range(g)})
        rest = [c for c in range(ncu) if c not in set(geo)]
        (gs, gh), (cs, ch) = _masked_stream(device, geo, ncu), _masked_stream(device, rest, ncu)
        _partitions[key] = (gs, cs, (gh, ch))
    return _partitions[key][:2]


class PipelinedForward:
    """``run(batches, extras=None)`` -> ``[model(x, *extra) for x, extra in ...]``, pipelined.

    geometry_cus: CUs reserved for the FPS chain (default 32: one per cloud of a B=32 batch)."""

    def __init__(self, model, geometry_cus=32):
        self.model = model
        self.geometry_cus = geometry_cus
        self.sas = [m for m in model.modules()
                    if isinstance(m, (PointNetSetAbstraction, PointNetSetAbstractionMsg))]

    def _fps_chain(self, x):
        """FPS of every SA layer for input x ([B, C, N]); draws in layer order."""
        entries = {}
        pts = x.permute(0, 2, 1)
        for sa in self.sas:
            if getattr(sa, "group_all", False):
                break
            B, N, _ = pts.shape
            _, newp, cpk, ppk = ops.fps_direct(pts, sa.point_number, shard.device_start(B, N, x.device))
            entries[id(sa)] = (pts.data_ptr(), newp, cpk, ppk)
            pts = newp
        return entries

    def run(self, batches, extras=None, post=None):
        """post(i, out) is called on the compute stream after batch i's forward (e.g. an
        all_gather of its logits)."""
        if self.model.training:
            raise RuntimeError("pn2.pipeline: eval mode only")
        if not batches:
            return []
        dev = batches[0].device
        geo, main = partition(dev.index, self.geometry_cus)
        caller = torch.cuda.current_stream(dev)
        geo.wait_stream(caller)
        main.wait_stream(caller)
        outs = []
        with torch.no_grad():
            with torch.cuda.stream(geo):
                nxt = self._fps_chain(batches[0])
                nxt_ev = geo.record_event()
            for i, x in enumerate(batches):
                entries, ev = nxt, nxt_ev
                if i + 1 < len(batches):  # batch i's draws were taken: take batch i+1's
                    with torch.cuda.stream(geo):
                        nxt = self._fps_chain(batches[i + 1])
                        nxt_ev = geo.record_event()
                main.wait_event(ev)
                for _, newp, cpk, ppk in entries.values():
                    for t in (newp, cpk, ppk):
                        t.record_stream(main)
                with torch.cuda.stream(main), geometry.provide(entries):
                    extra = () if extras is None else tuple(extras[i])
                    out = self.model(x, *extra)
                    if post is not None:
                        out = post(i, out)
                if entries:
                    raise RuntimeError("pn2.pipeline: the model did not consume every "
                                       "precomputed FPS (SA layers called out of order?)")
                outs.append(out)
        caller.wait_stream(main)
        caller.wait_stream(geo)
        return outs
