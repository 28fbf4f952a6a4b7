"""Pipelined eval forward over a stream of batches.

Every SA layer's farthest point sampling depends only on the point coordinates (sa1 samples the
input cloud, sa2 the centroids sa1 chose, ...), never on an MLP output, so a batch's whole FPS
chain can run before its forward.  The pipeline runs the FPS chain of batch i+1 on a
*geometry* stream while the ball queries and MLPs of batch i run on a *compute* stream: FPS is a
serial, latency-bound loop of one workgroup per cloud (32 workgroups at B=32) that leaves
almost all of the chip idle, so overlapping it takes it off the critical path.

``GraphedPipeline`` (the launch bench.py uses) replays every stage from HIP graphs; the eager
``PipelinedForward`` issues ~25 launches per batch from Python, ~470 us of host time at SSG
B=32, which is longer than the compute stream's work once the MLP kernels are fast.

CUs.  By default (geometry_cus=0) the streams are ordinary streams sharing every CU, geometry
at high priority.  ``geometry_cus > 0`` gives the geometry stream its own CUs instead
(hipExtStreamCreateWithCUMask through pn2_stream_create_cu_masked; see ``_streams`` for how
MI355X maps mask bits to XCDs).  Measured, SSG B=32 N=1024, graphed: shared 69.5k / 69.9k
clouds/s; 8 dedicated CUs (1 per XCD) 65.0k / 65.1k; 24 CUs 63.3k / 64.4k -- FPS co-resident
with the MFMA kernels costs the chains less than the CUs a partition withholds from them.

The tail of each forward -- everything after the last SA layer returns (the FC head, `post`;
in ``GraphedPipeline`` also a trailing group_all layer, see ``_split_index``) -- can run on a
third stream: it is a dozen tiny launches (the head's largest GEMM has 2
workgroups) that would otherwise sit on the compute stream between batch i's last MLP and batch
i+1's first.  The switch is a forward hook on the last SA module, active only inside ``run``.
The last SA layer's outputs are handed over with ``record_stream``; any other compute-stream
tensor the tail reads (e.g. the translation heads' ``mean``, computed before sa1 and added
after the head) would not be, so ``tail="auto"`` uses it only for models called without extra
inputs (every reference head but translation_*); ``tail=True`` forces it.  Off by default in
the eager pipeline (its host issue time is the bound there: 62.6k vs 66.0k clouds/s measured),
on in ``GraphedPipeline``, whose static buffers make it safe for every head.

Results and RNG.  Every batch computes what ``model(x)`` computes: the SA layers run the same
kernels and produce the same bits (test_pipelined_forward_matches_eager); the head's own
``nn.Linear`` layers go through torch's BLAS, which may choose a different GEMM kernel on
another stream (last-ulp differences in logits).  The reference draws one ``torch.randint(0, N, (B,))`` per SA layer from the CPU
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
import contextlib
import os
import time

import torch

from . import _lib
from . import geometry
from . import ops
from . import shard
from . import tuning
from .pointnet2_utils import PointNetSetAbstraction, PointNetSetAbstractionMsg, msg_ball_queries

_partitions = {}  # (device, geometry CUs) -> (geometry, compute, tail streams, raw handles)


@atexit.register
def _destroy_partitions():
    """Release the CU-masked streams before the HIP runtime tears down (left to process exit,
    their destruction raced the runtime's own teardown under rocprofv3)."""
    for key, (*_, raw) in list(_partitions.items()):
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


# hipExtStreamCreateWithCUMask on MI355X (measured, tools/micro/cu_mask_map.hip): mask bit i
# belongs to XCD i % 8 and selects CU i / 8 of it, and an XCD whose share of the mask is empty
# is NOT restricted (all 32 of its CUs run the stream).  So a partition is a contiguous block of
# bits: [0, g) = g/8 CUs on every XCD, [g, 256) = the other CUs of every XCD.  (A mask spread
# with stride 8 -- bits 0, 8, 16, ... -- is XCD 0 alone plus the seven unrestricted XCDs: the
# whole chip.)
_XCDS = 8


_extra = {}  # device -> (second geometry stream, second compute stream)


def _hw_queues():
    """Hardware queues per process the HIP runtime was started with (GPU_MAX_HW_QUEUES)."""
    try:
        return max(1, int(os.environ.get("GPU_MAX_HW_QUEUES", "4")))
    except ValueError:
        return 4


def _streams(device, geometry_cus):
    key = (device, geometry_cus)
    if key not in _partitions and int(geometry_cus) <= 0:
        # no partition: ordinary streams sharing every CU, geometry at high priority.  A HIP
        # stream is bound to one of the process's hardware queues at its first command (up to
        # GPU_MAX_HW_QUEUES = 4 per priority; past that, the least-used one).  Which queue a
        # pipeline stream lands on changed the throughput by up to 45 % (SSG, rocprofv3
        # Queue_Id per dispatch, tools/debug/gpipe_events.py): with the default stream's queue
        # first, the streams first used second and third ran at full speed, while a stream on
        # the fourth queue fell behind -- the tail stream there took 570-800 us per head
        # instead of 130-300 (58-65k clouds/s), the second compute stream there cost ~8 %
        # (97-100k), and a stream first used late (after the captures' streams) shared another
        # pipeline stream's queue (84-87k).  So the geometry, first compute and tail streams
        # each run one tiny command here, in that order, and the second compute stream is the
        # default stream itself, whose queue exists from the start: 103-106k at any slot count.
        dev = torch.device("cuda", device)
        lo, hi = torch.cuda.Stream.priority_range()
        geo = torch.cuda.Stream(dev, priority=min(lo, hi))
        geo2 = torch.cuda.Stream(dev, priority=min(lo, hi))
        main = torch.cuda.Stream(dev)
        # tuning tail_prio = 1: the tail (heads) at high priority as well (A/B)
        tail = torch.cuda.Stream(dev, priority=min(lo, hi) if tuning.get("tail_prio") else 0)
        main2 = torch.cuda.default_stream(dev)
        tail2 = torch.cuda.Stream(dev, priority=min(lo, hi) if tuning.get("tail_prio") else 0)
        # one more normal-priority stream, never used: creating it moves the hardware queues
        # the later geometry streams (_extra_geometry_streams) get, and without it the headline
        # pipeline loses 15-25 % (r06, same box, interleaved: K = 20 117-122k with it, 88-99k
        # without; tools/ab_worktree.sh)
        spare = torch.cuda.Stream(dev)
        for st in (geo, main, tail):
            with torch.cuda.stream(st):
                torch.zeros(1, device=dev)
            st.synchronize()
        _partitions[key] = (geo, main, tail, ())
        _extra[device] = (geo2, main2, tail2, spare)
    if key not in _partitions:
        ncu = _cu_count(device)
        per = max(1, min(int(geometry_cus) // _XCDS, ncu // _XCDS - 1))  # CUs per XCD
        geo = list(range(per * _XCDS))
        rest = list(range(per * _XCDS, ncu))
        (gs, gh), (cs, ch) = _masked_stream(device, geo, ncu), _masked_stream(device, rest, ncu)
        ts, th = _masked_stream(device, geo, ncu)
        _partitions[key] = (gs, cs, ts, (gh, ch, th))
    return _partitions[key][:3]


_more_geo = {}  # device -> geometry streams past the second (GraphedPipeline(geometry_streams>2))


def _extra_geometry_streams(device, n):
    """n (0-3) more high-priority streams for GraphedPipeline(geometry_streams=1+n) (shared
    CUs; the second is created with the others by _streams, later ones on first use).  n = 0
    touches no stream: with geometry_cus > 0 the shared-CU set would add queues beyond the
    masked streams'."""
    if n <= 0:
        return []
    _streams(device, 0)
    more = _more_geo.setdefault(device, [])
    while len(more) < n - 1:
        lo, hi = torch.cuda.Stream.priority_range()
        st = torch.cuda.Stream(torch.device("cuda", device), priority=min(lo, hi))
        with torch.cuda.stream(st):
            torch.zeros(1, device=torch.device("cuda", device))
        st.synchronize()
        more.append(st)
    return ([_extra[device][0]] + more)[:n]


def _extra_compute_streams(device, n):
    """n (0 or 1) more compute streams for GraphedPipeline(compute_streams=1+n) (created with
    the others by _streams): the process's default stream."""
    if n <= 0:
        return []
    _streams(device, 0)
    return [_extra[device][1]][:n]


def partition(device, geometry_cus):
    """(geometry stream, compute stream) on `device`: `geometry_cus` CUs (rounded down to a
    multiple of the XCD count, at least one per XCD) for the FPS chain, all the others for
    everything else.  Cached per (device, count)."""
    return _streams(device, geometry_cus)[:2]


class PipelinedForward:
    """``run(batches, extras=None)`` -> ``[model(x, *extra) for x, extra in ...]``, pipelined.

    geometry_cus: 0 (default): streams share every CU; > 0: CUs reserved for the FPS chain.
    tail: run what follows the last SA layer (head, `post`) on the geometry CUs: False
    (default), "auto" (when `run` gets no extras) or True."""

    def __init__(self, model, geometry_cus=0, tail=False):
        self.model = model
        self.geometry_cus = geometry_cus
        self.tail = tail
        self.sas = self._find_sas()

    def _find_sas(self):
        return [m for m in self.model.modules()
                if isinstance(m, (PointNetSetAbstraction, PointNetSetAbstractionMsg))]

    _GEO_ATTRS = ("point_number", "sample_number", "radius", "group_all", "radius_list",
                  "sample_number_list")

    def _geo_sig(self):
        """What the geometry graphs bake in besides the input: each SA module and its sampling /
        grouping configuration (an in-place change of e.g. ``sa1.radius`` must recapture)."""
        def frz(v):
            return tuple(v) if isinstance(v, list) else v
        return tuple((id(sa),) + tuple(frz(getattr(sa, a, None)) for a in self._GEO_ATTRS)
                     for sa in self.sas)

    @staticmethod
    def _to_tail(tail):
        """Forward hook for the last SA module: hand its outputs to the tail stream and make it
        current for the rest of the forward."""
        def hook(module, inputs, output):
            main = torch.cuda.current_stream()
            tail.wait_stream(main)
            for t in output if isinstance(output, (tuple, list)) else (output,):
                if isinstance(t, torch.Tensor):
                    t.record_stream(tail)
            torch.cuda.set_stream(tail)
        return hook

    def _fps_chain(self, x):
        """Geometry of every SA layer for input x ([B, C, N]): FPS (draws in layer order) and
        the ball query of each radius -- both read only coordinates, so a batch's whole
        geometry runs ahead of its MLPs.  A group_all layer ends a head's chain; an SA layer
        after it starts the next head's chain from the input again (a model holding several
        heads over the same cloud, e.g. MultiHead(rotation_ssg, translation_ssg)).

        Several chains: their first layers all sample the input, so they run as ONE FPS launch
        over the input repeated once per chain (each copy with its own start draws).  FPS is
        latency-bound on one workgroup per cloud -- 16 clouds take as long as 8
        (tools/debug/fps_batch_merge.py) -- so the heads' first FPS run side by side instead of
        one after the other.  The copy keeps x's layout (the packed squared norms follow the
        reference's layout-dependent summation order), and every start is still drawn in layer
        order before any launch."""
        with self._profile():  # the launch choices measured best beside the chains
            return self._fps_chain_body(x)

    def _profile(self):
        """The kernel-selection profile of this pipeline's launches: tuning.PIPELINE_PROFILE
        where it was measured best -- the eager pipeline, and graphed pipelines whose launches
        carry >= 64 clouds (four fused B=32 batches, where r05 tuned it; STRESS's B=128; POSE's
        two heads over B=64: 71-72k vs 68-70k) -- else the eager forward's defaults (graphed SSG
        at one B=32 batch per launch: 104-112k vs 97-100k clouds/s with the profile, K = 20,
        interleaved x3; MSG flat).  Host key pipe_profile: 0 never, 2 always."""
        mode = int(tuning.get("pipe_profile"))
        if mode == 2 or (mode == 1 and getattr(self, "launch_batch", 128) >= 64):
            return tuning.pipeline_profile()
        return contextlib.nullcontext()

    def _fps_chain_body(self, x):
        B, _, N = x.shape
        dev = x.device
        chains, cur = [], []
        for sa in self.sas:
            if getattr(sa, "group_all", False):
                if cur:
                    chains.append(cur)
                cur = []
                continue
            cur.append(sa)
        if cur:
            chains.append(cur)
        starts = {}  # drawn in layer order, as the eager forwards draw them
        for ch in chains:
            n = N
            for sa in ch:
                starts[id(sa)] = shard.device_start(B, n, dev)
                n = sa.point_number
        entries = {}
        # geometry_bq = 0: the ball queries run in each batch's forward instead (the module
        # queries when its entry holds no lists), leaving the FPS alone on the geometry stream
        gbq = getattr(self, "geometry_bq", None)
        bq = bool(tuning.get("geometry_bq")) if gbq is None else bool(gbq)
        pts = x.permute(0, 2, 1)
        first = {}  # chain -> (newp, cpk, ppk) of its first layer
        heads = [ch[0] for ch in chains]
        merge = len(chains) > 1 and len({sa.point_number for sa in heads}) == 1 and \
            (pts.stride(2) == 1 or x.stride(2) == 1)
        if merge:
            k = len(chains)
            # the same strides as pts: rows-contiguous stays rows, channel-first stays that
            rep = torch.cat([pts] * k) if pts.stride(2) == 1 else torch.cat([x] * k).permute(0, 2, 1)
            _, newp, cpk, ppk = ops.fps_direct(rep, heads[0].point_number,
                                               torch.cat([starts[id(sa)] for sa in heads]))
            for i, ch in enumerate(chains):
                first[i] = (newp[i * B:(i + 1) * B], cpk[i * B:(i + 1) * B], ppk[i * B:(i + 1) * B])
        for i, ch in enumerate(chains):
            p = pts
            for j, sa in enumerate(ch):
                C = p.shape[2]
                if j == 0 and i in first:
                    newp, cpk, ppk = first[i]
                else:
                    _, newp, cpk, ppk = ops.fps_direct(p, sa.point_number, starts[id(sa)])
                if not bq:
                    idxs = []
                elif isinstance(sa, PointNetSetAbstractionMsg):
                    idxs = msg_ball_queries(ppk, cpk, C, sa.radius_list, sa.sample_number_list)
                else:
                    idxs = [ops.ball_query_direct(ppk, cpk, C, sa.radius, sa.sample_number, True)]
                entries[id(sa)] = (p.data_ptr(), newp, cpk, ppk, idxs)
                p = newp
        return entries

    def run(self, batches, extras=None, post=None):
        """post(i, out) is called on the compute stream after batch i's forward (e.g. an
        all_gather of its logits)."""
        return self._run_eager(batches, extras, post, self.tail)

    def _run_eager(self, batches, extras, post, tail):
        if self.model.training:
            raise RuntimeError("pn2.pipeline: eval mode only")
        if not batches:
            return []
        dev = batches[0].device
        geo, main, tail = _streams(dev.index, self.geometry_cus)
        caller = torch.cuda.current_stream(dev)
        geo.wait_stream(caller)
        main.wait_stream(caller)
        tail.wait_stream(caller)
        outs = []
        handle = None
        use_tail = (extras is None) if tail == "auto" else bool(tail)
        if use_tail and self.sas:
            handle = self.sas[-1].register_forward_hook(self._to_tail(tail))
        try:
            with self._profile():
                self._run(batches, extras, post, geo, main, outs)
        finally:
            if handle is not None:
                handle.remove()
        caller.wait_stream(main)
        caller.wait_stream(geo)
        caller.wait_stream(tail)
        return outs

    def _run(self, batches, extras, post, geo, main, outs):
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
                for _, newp, cpk, ppk, idxs in entries.values():
                    for t in [newp, cpk, ppk] + [t for ic in idxs for t in ic]:
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


class MultiHead(torch.nn.Module):
    """Several heads over the same input as one module, so the pipeline overlaps all of their
    geometry with all of their MLPs: forward(x, *extras) -> tuple of each head's output, the
    heads called in order (their FPS draws in that order, as separate eager calls take them).
    extra_heads: indices of the heads that also take the extras (translation heads' mean)."""

    def __init__(self, heads, extra_heads=()):
        super().__init__()
        self.heads = torch.nn.ModuleList(heads)
        self.extra_heads = set(extra_heads)
        self.training = any(h.training for h in heads)  # the heads' mode, unchanged

    def forward(self, x, *extras):
        return tuple(h(x, *extras) if i in self.extra_heads else h(x)
                     for i, h in enumerate(self.heads))


def _clone(o):
    if isinstance(o, torch.Tensor):
        return o.clone()
    if isinstance(o, (tuple, list)):
        return type(o)(_clone(t) for t in o)
    return o


def _rows(o, lo, hi):
    """Rows [lo, hi) (dim 0) of every tensor of a (nested) output: batch h of a fused group's."""
    if isinstance(o, torch.Tensor):
        return o[lo:hi]
    if isinstance(o, (tuple, list)):
        return type(o)(_rows(t, lo, hi) for t in o)
    return o


def _flat_tensors(o):
    if isinstance(o, torch.Tensor):
        return [o]
    if isinstance(o, (tuple, list)):
        return [t for x in o for t in _flat_tensors(x)]
    return []


# thread-local capture: other threads (the RCCL watchdog of a multi-GPU run) may keep querying
# their own events while a pipeline slot is captured
_MODE = "thread_local"


class _Slot:
    """Static buffers and graphs of one batch slot: one batch of a geometry group, or the whole
    group (``fused``)."""
    fused = False


class _Restart(Exception):
    """An SA module was replaced between runs: the geometry graphs are stale (run() restarts)."""


class _Group:
    """Static inputs and the geometry graph of ``geometry_batches`` consecutive batches; its
    ``halves`` are their batch slots."""


def _batched_like(x, n):
    """An uninitialised [n * B, ...] tensor whose every [B, ...] slice has x's strides (so a
    cloud keeps its memory layout, on which the reference's summation orders depend), or None
    when the batch is not x's outermost dimension."""
    order = sorted(range(x.dim()), key=lambda d: (-x.stride(d), d))
    if order[0] != 0:
        return None
    shape = [x.shape[d] for d in order]
    shape[0] *= n
    buf = torch.empty(shape, dtype=x.dtype, device=x.device)
    inv = [order.index(d) for d in range(x.dim())]
    return buf.permute(inv)


class GraphedPipeline(PipelinedForward):
    """``PipelinedForward`` with every stage replayed from HIP graphs: no per-kernel host work.

    The eager pipeline issues ~25 launches plus the SA modules' Python per batch; on MI355X that
    host time (~0.5 ms per SSG B=32 batch) is as long as the GPU work, so the GPU idles.  Here
    batches are taken in *groups* of ``geometry_batches`` consecutive batches; each of the
    ``nslots // geometry_batches`` group slots (group g uses slot g % groups) holds static
    inputs for its batches and one captured geometry graph, and each of its batch slots two
    forward graphs:
      fps   the group's geometry (``_fps_chain`` over the group's batches side by side: FPS +
            ball queries), replayed on a geometry stream ``groups - 1`` groups ahead of the
            compute stream;
      sa    a batch's forward up to the last SA layer, replayed on the compute stream;
      head  the rest of the forward, replayed on a third stream (``tail``; with tail=False,
            head is part of sa).
    Each batch's forward reads its own slice of the group's geometry, so it computes exactly
    what its own eager forward computes (per-cloud kernels; the FC tail's row kernel computes a
    row the same way at any row count).  The capture is split by a forward hook
    (capture_end / capture_begin) after the last SA layer that groups neighbourhoods
    (``_split_index``: a trailing group_all layer goes with the head; the eager
    ``PipelinedForward`` tail still splits after the last SA layer).

    Why groups: FPS is a serial, latency-bound loop on one workgroup per cloud, so a launch
    over 2B clouds takes about what one over B clouds takes.  Under the MLP kernels' contention
    one SSG B=32 batch's FPS chain took 690-770 us (tools/debug/gpipe_events.py) against a
    ~300 us compute period: with one batch per geometry replay and two geometry streams the
    pipeline was geometry-bound at ~375 us per batch.  Two batches per replay halve that.

    Events order the slot reuse: group g+groups's fps waits until group g's batches' sa and head
    graphs and output clones have run (it overwrites the group's inputs and geometry outputs,
    which a group_all layer in a head graph still reads); a batch's sa waits for the head of
    the batch that used its batch slot before (they share a memory pool).

    RNG and results: as PipelinedForward.  The first batch of a new input signature (or after
    any parameter change) runs through the eager pipeline -- its real result, its draws -- and
    every slot is captured after it; the captures draw nothing.  Every replayed batch takes its
    draws on the host in batch order (shard.draw_start, so shard.batch_shard applies) into its
    part of the group's start buffer, uploaded before the group's fps replay.  A last group
    with fewer batches repeats its first batch's input in the empty places (no draws, results
    unused).  Outputs are cloned out of the static buffers on the stream that produced them.

    compute_streams=2 (default with shared CUs): consecutive batches' sa graphs alternate
    between two compute streams, so one batch's short dependent kernels (scans, the pre-pass)
    and its kernels' last partial waves of workgroups run beside the other batch's chains.
    geometry_streams=2..4: consecutive groups' geometry replays alternate between that many
    high-priority streams.  A process gets 4 hardware queues (GPU_MAX_HW_QUEUES): one geometry
    stream + two compute streams + the tail stream is the default; with two geometry streams
    and two compute streams the head graphs run on their batch's compute stream after its sa
    graph (no tail stream).  Measured (SSG B=32, 100 batches, clouds/s): 1 compute + 2 geometry
    streams, 6 slots 95-96.7k; 2 compute + 1 geometry + tail, 8 slots 106-107k (MSG +12.6 %,
    POSE +7.9 %, STRESS +2.8 %); 2 + 2, head on the compute streams, 8 slots 103-104k.  The slot
    count matters beyond "enough": 2 + 1 at 4 / 6 / 8 / 12 / 16 slots gave 92 / 100 / 107 /
    91 / 106k (unexplained; reproducible per count).
    """

    def __init__(self, model, geometry_cus=0, tail=True, nslots=16, geometry_streams=1,
                 geometry_batches=4, compute_streams=None, fuse=None, geometry_bq=None,
                 tail_streams=None):
        super().__init__(model, geometry_cus, bool(tail))
        # geometry_bq: the ball queries on the geometry streams after each layer's FPS (True),
        # or in each batch's forward on the compute streams (False); None: tuning geometry_bq
        self.geometry_bq = geometry_bq
        # fuse: one forward (sa + head graphs) over the whole geometry group -- its gb batches
        # side by side, every launch with gb times the rows -- instead of one per batch.  Each
        # cloud is computed exactly as in its own batch's forward (per-cloud kernels; the FC
        # tail computes a row the same way at any row count), so the outputs are the per-batch
        # ones, sliced.  Default: tuning pipe_fuse.
        self.fuse = bool(tuning.get("pipe_fuse")) if fuse is None else bool(fuse)
        gb = int(geometry_batches)
        if gb < 1:
            raise ValueError("pn2.pipeline: geometry_batches must be >= 1")
        if nslots < 2 * gb or nslots % gb:
            raise ValueError("pn2.pipeline: GraphedPipeline needs nslots a multiple of "
                             "geometry_batches and at least two groups")
        if geometry_cus > 0:
            geometry_streams = 1  # the CU-partitioned geometry stream is one
        # 2 at most: with the compute and tail streams that is the 4 hardware queues a process
        # gets (GPU_MAX_HW_QUEUES); a fifth stream shares a queue and serialises behind another
        # (measured: 3 geometry streams 42.8k clouds/s at SSG vs 76.1k with 2)
        if geometry_streams not in (1, 2, 3, 4):
            raise ValueError("pn2.pipeline: geometry_streams is 1 to 4")
        if compute_streams is None:
            compute_streams = 2 if geometry_cus <= 0 else 1
        if compute_streams not in (1, 2):
            raise ValueError("pn2.pipeline: compute_streams is 1 or 2")
        if compute_streams > 1 and geometry_cus > 0:
            raise ValueError("pn2.pipeline: compute_streams > 1 needs shared CUs (geometry_cus=0)")
        self.compute_streams = int(compute_streams)
        # the head graphs get the tail stream(s) while the process's hardware queues allow it
        # (GPU_MAX_HW_QUEUES, HIP's default 4; bench.py runs with 8): every stream on a queue
        # of its own
        ts = int(tuning.get("tail_streams")) if tail_streams is None else int(tail_streams)
        self.tail_streams = 2 if ts == 2 and geometry_cus <= 0 else 1
        self.head_on_tail = (geometry_streams + self.compute_streams + self.tail_streams <= _hw_queues() and
                             not tuning.get("heads_on_compute"))  # A/B
        self.nslots = int(nslots)
        self.gb = gb
        self.ngroups = self.nslots // gb
        self.geometry_streams = int(geometry_streams)
        self.trace = None
        self._key = None  # (input signature, precision) the slots were captured for
        self._params = None  # graphs.ParamState of the model
        self._pkey = None  # its key at the last capture
        self._slots = None  # the group slots

    def _split_index(self):
        """The SA module after which a slot's compute graph ends and its tail graph begins.  The
        last SA layer when it groups neighbourhoods; when it is a group_all layer (sa3 of every
        reference head: M = B rows, a few hundred workgroups, latency-bound), the layer before
        it, so the group_all layer runs with the head on the tail stream -- beside the next
        batch's wide sa1/sa2 kernels instead of after them.  Only with shared CUs: with
        geometry_cus > 0 the tail stream is masked to the geometry CUs, where a group_all MLP
        would compete with FPS on a few CUs.  Tuning pipe_split_last = 1 keeps the old split (A/B).

        The head graph then reads the split layer's outputs -- sa2's centroids are a static
        output of the group's fps graph -- so the group's next fps replay waits for the head
        (``ev_read`` in ``run``), not only for the sa graph."""
        k = len(self.sas) - 1
        if (k > 0 and getattr(self.sas[k], "group_all", False) and self.geometry_cus <= 0 and
                not tuning.get("pipe_split_last")):
            k -= 1
        return k

    def _capture(self, x, extra, dev, draws):
        gb, B = self.gb, x.shape[0]
        grp = _Group()
        grp.x = _batched_like(x, gb) if gb > 1 else None
        if grp.x is None:
            if gb > 1:
                raise RuntimeError("pn2.pipeline: geometry_batches > 1 needs the batch as the "
                                   "input's outermost dimension")
            grp.x = x.clone()
        grp.x.copy_(torch.cat([x] * gb) if gb > 1 else x)
        xs = [grp.x[h * B:(h + 1) * B] for h in range(gb)]
        # the start buffer exists before the capture: allocated inside it, it could share pool
        # memory with a temporary the capture freed earlier, which the replay rewrites after
        # the buffer was uploaded.  Layout: per draw d of a batch (layer order), a block of
        # gb * B_d starts, batch h of the group at [h * B_d, (h + 1) * B_d) of the block.
        grp.start_buf = torch.empty(gb * sum(b for b, _ in draws), dtype=torch.long, device=dev)
        blocks, off = [], 0
        for b, n in draws:
            blocks.append((grp.start_buf[off:off + gb * b], gb * b, n))
            off += gb * b
        it = iter(blocks)

        def static_start(Bq, Nq, device):
            t, b, n = next(it)
            if (b, n) != (Bq, Nq):
                raise RuntimeError("pn2.pipeline: FPS draw shapes changed during capture")
            return t

        grp.fps = torch.cuda.CUDAGraph()
        fps_pool = torch.cuda.graph_pool_handle()
        cs = torch.cuda.Stream(dev)
        torch.cuda.synchronize(dev)
        with torch.no_grad(), torch.cuda.stream(cs), shard.start_source(static_start):
            grp.fps.capture_begin(pool=fps_pool, capture_error_mode=_MODE)
            entries = self._fps_chain(grp.x)
            grp.fps.capture_end()
        torch.cuda.synchronize(dev)
        grp.entries = entries
        grp.B = B
        grp.halves = self._group_forwards(grp, xs, extra, dev)
        return grp

    def _group_forwards(self, grp, xs, extra, dev):
        """The group's forward graphs: one per batch, or (fuse) one over the whole group."""
        gb = self.gb
        if self.fuse and gb > 1:
            ex = [torch.cat([e] * gb) for e in extra]
            sl = self._capture_forward(grp.x, ex, dev, *self._half_entries(grp, None))
            outs = _flat_tensors(sl.out)
            if outs and all(t.dim() >= 1 and t.shape[0] == gb * grp.B for t in outs):
                sl.fused = True
                return [sl]
            # an output without the batch as its first dimension: per-batch forwards
        return [self._capture_forward(xs[h], extra, dev, *self._half_entries(grp, h))
                for h in range(gb)]

    def _half_entries(self, grp, h):
        """Batch h's slice of the group's geometry, keyed by the tensor its SA module is called
        with in that batch's forward (its slice of the input or of the previous layer's
        centroids), and the storages of the group's geometry outputs."""
        B = grp.B
        srcs = {grp.x.data_ptr(): grp.x}
        for _, newp, _, _, _ in grp.entries.values():
            srcs[newp.data_ptr()] = newp

        def part(t):  # h None: the whole group (a fused forward)
            return t if h is None else t[h * B:(h + 1) * B]

        geo = set()
        for _, newp, cpk, ppk, idxs in grp.entries.values():
            geo.update(t.untyped_storage().data_ptr()
                       for t in [newp, cpk, ppk] + [t for ic in idxs for t in ic])
        ent = {k: (part(srcs[ptr]).data_ptr(), part(newp), part(cpk), part(ppk),
                   [tuple(part(t) for t in ic) for ic in idxs])
               for k, (ptr, newp, cpk, ppk, idxs) in grp.entries.items()}
        return ent, geo

    def _recapture_forwards(self, extra, dev):
        """New sa / head graphs for every batch slot after a parameter change (their kernels
        read the parameters' memory); the geometry graphs read only coordinates and draws, and
        are kept."""
        with self._profile():
            for grp in self._slots:
                B = grp.B
                grp.halves = self._group_forwards(
                    grp, [grp.x[h * B:(h + 1) * B] for h in range(self.gb)], extra, dev)

    def _capture_forward(self, x, extra, dev, entries, geo):
        sl = _Slot()
        sl.x = x
        sl.extra = tuple(e.clone() for e in extra)
        sl.sa = torch.cuda.CUDAGraph()
        sl.head = torch.cuda.CUDAGraph() if self.tail else None
        fwd_pool = torch.cuda.graph_pool_handle()

        def split(module, inputs, output):
            sl.sa.capture_end()
            sl.sa_out = output
            sl.head.capture_begin(pool=fwd_pool, capture_error_mode=_MODE)

        cs = torch.cuda.Stream(dev)
        torch.cuda.synchronize(dev)
        handle = self.sas[self._split_index()].register_forward_hook(split) if self.tail else None
        try:
            with torch.no_grad(), torch.cuda.stream(cs):
                sl.sa.capture_begin(pool=fwd_pool, capture_error_mode=_MODE)
                with geometry.provide(dict(entries)):
                    sl.out = self.model(sl.x, *sl.extra)
                (sl.head if self.tail else sl.sa).capture_end()
        finally:
            if handle is not None:
                handle.remove()
        torch.cuda.synchronize(dev)
        # does anything after the sa graph read the geometry graph's outputs?  The head graph
        # does when it holds a layer (a trailing group_all reads the split layer's centroids);
        # the output clone does when the model returns one of them
        outs = sl.out if isinstance(sl.out, (tuple, list)) else (sl.out,)
        flat = [t for o in outs for t in (o if isinstance(o, (tuple, list)) else (o,))]
        sl.tail_reads_geometry = (self.tail and self._split_index() < len(self.sas) - 1) or any(
            isinstance(t, torch.Tensor) and t.untyped_storage().data_ptr() in geo for t in flat)
        return sl

    def run(self, batches, extras=None, post=None):
        if self.model.training:
            raise RuntimeError("pn2.pipeline: eval mode only")
        if not batches:
            return []
        extra_of = (lambda i: ()) if extras is None else (lambda i: tuple(extras[i]))
        from .graphs import ParamState, _sig
        x0, e0 = batches[0], extra_of(0)
        sig = (_sig((x0,) + tuple(e0)), ops.current_precision(), self._geo_sig())
        # the other batches need only the same input signature; a batch list repeating one
        # input needs nothing
        for i in range(1, len(batches)):
            x = batches[i]
            if x is x0 and (extras is None or all(a is b for a, b in zip(extra_of(i), e0))):
                continue
            if _sig((x,) + extra_of(i)) != sig[0]:
                return self._run_eager(batches, extras, post, False)  # mixed shapes: eager
        if self._params is None:
            self._params = ParamState(self.model)
        outs, first = [], 0
        dev = batches[0].device
        # clouds per launch (PipelinedForward._profile)
        self.launch_batch = int(x0.shape[0]) * (self.gb if self.fuse else 1)
        # With the same input signature the parameters (the sa / head graphs read their memory)
        # are checked only after the first geometry group is issued: the geometry graphs read
        # coordinates and draws alone, and the check's host time (a walk over every parameter
        # and buffer, ~40-110 us) then overlaps that group's FPS instead of delaying it.
        check_params = self._slots is not None and sig == self._key
        rng0 = shard.rng_state() if check_params else None  # see the parameter check below
        if not check_params:
            self.sas = self._find_sas()
            sig = sig[:2] + (self._geo_sig(),)
            self._slots = None
            draws = []

            def record(B, N, device):
                draws.append((B, N))
                return shard.draw_start(B, N).to(device, non_blocking=True)

            with shard.start_source(record):
                outs = self._run_eager(batches[:1], None if extras is None else extras[:1],
                                       post, False)
            self._draws = draws
            with self._profile():
                self._slots = [self._capture(batches[0], extra_of(0), dev, draws)
                               for _ in range(self.ngroups)]
            self._key = sig
            self._pkey = self._params.key()  # capture allocations do not touch parameters
            # replay every captured graph once now, in dependency order on this stream (start
            # index 0: a valid point; outputs land in static buffers that real replays
            # overwrite; no RNG inside the graphs): a graph's first launch costs extra, and
            # otherwise the slots a short first run does not reach pay it in the next one
            for grp in self._slots:
                grp.start_buf.zero_()
                grp.fps.replay()
                for sl in grp.halves:
                    sl.sa.replay()
                    if sl.head is not None:
                        sl.head.replay()
            torch.cuda.synchronize(dev)
            first = 1
        if first == len(batches):
            return outs
        gb, ng = self.gb, self.ngroups
        nbat = len(batches) - first
        ngr = (nbat + gb - 1) // gb  # groups this call
        geo, main, tail = _streams(dev.index, self.geometry_cus)
        geos = [geo] + _extra_geometry_streams(dev.index, self.geometry_streams - 1)
        mains = [main] + _extra_compute_streams(dev.index, self.compute_streams - 1)
        tails = [tail] + ([_extra[dev.index][2]] if self.tail_streams == 2 else [])
        caller = torch.cuda.current_stream(dev)
        ev0 = caller.record_event()  # one event for every pipeline stream to wait on
        for st in geos + mains + tails:
            st.wait_event(ev0)
        # per group slot: the fps replay's event, and the events after which the group's
        # batches no longer read its inputs / geometry (one per batch: with two compute
        # streams they finish on different streams)
        ev_fps, ev_read = [None] * ng, [[] for _ in range(ng)]
        ev_head = [None] * (ng * gb)  # per batch slot
        starts = self._draw_all(ngr)

        tr = self.trace  # optional list of per-batch timing events (tools/debug/gpipe_events.py)

        def mark(j, name, stream):
            if tr is not None:
                while len(tr) <= j:
                    tr.append({})
                e = torch.cuda.Event(enable_timing=True)
                e.record(stream)
                tr[j][name] = (e, time.perf_counter())

        def issue_fps(g):
            s = g % ng
            grp = self._slots[s]
            geo = geos[g % len(geos)]
            js = [first + g * gb + h for h in range(gb)]
            nh = sum(1 for j in js if j < len(batches))
            with torch.cuda.stream(geo):
                # the group slot's previous batches are done with its inputs and geometry
                # outputs: their sa graphs read them, and so did their head graphs when the
                # split put a group_all layer there (sa3 reads sa2's centroids)
                for e in ev_read[s]:
                    geo.wait_event(e)
                ev_read[s] = []
                mark(js[0] - first, "geo0", geo)
                for h, j in enumerate(js):
                    grp.x[h * grp.B:(h + 1) * grp.B].copy_(batches[j if j < len(batches) else js[0]],
                                                           non_blocking=True)
                grp.start_buf.copy_(self._draw_row(starts, g, nh), non_blocking=True)
                grp.fps.replay()
                ev_fps[s] = geo.record_event()
                mark(js[0] - first, "geo1", geo)

        drain = int(tuning.get("drain_heads"))  # see the head stream choice below
        issued = [0]  # geometry groups issued so far (always in group order: the draw order)

        def top_up(force, limit):
            # every group <= force now (a batch's own group), then at most one more while it
            # stays <= limit: group j takes the slot of group j - ng, so it waits until that
            # group's batches are all issued (their ev_read events exist).  One group per batch
            # interleaves the host's geometry issue with the compute issue, so the first batch's
            # sa graph is issued right behind its geometry, not behind ng-1 groups of it
            while issued[0] <= min(force, ngr - 1):
                issue_fps(issued[0])
                issued[0] += 1
            if issued[0] <= min(limit, ngr - 1):
                issue_fps(issued[0])
                issued[0] += 1

        if self._slots[0].halves[0].fused:
            try:
                with torch.no_grad():
                    self._run_fused(batches, extra_of, post, first, outs, ngr, geos, mains, tails,
                                    tail, ev_fps, ev_read, ev_head, top_up, check_params, dev, mark)
            except _Restart:
                torch.cuda.synchronize(dev)
                shard.set_rng_state(rng0)
                self._slots = None
                return self.run(batches, extras, post)
            for g in geos[1:]:
                geo.wait_stream(g)
            self._pinned_evs[self._pinned_cur] = geo.record_event()  # uploads read it
            for st in [geo] + mains + tails:
                caller.wait_stream(st)
            return outs
        with torch.no_grad():
            # the geometry runs up to ng-1 groups ahead of the compute streams
            for i in range(first, len(batches)):
                g, h = divmod(i - first, gb)
                s = g % ng
                bs = s * gb + h
                top_up(g, -1)
                if check_params:  # (first batch: its group's geometry is issued)
                    check_params = False
                    pk = self._params.key()
                    if pk != self._pkey:
                        if [id(m) for m in self._find_sas()] != [id(m) for m in self.sas]:
                            # an SA module was replaced: the geometry graphs are stale too.
                            # Take back the issued group's draws and start over (full capture)
                            torch.cuda.synchronize(dev)
                            shard.set_rng_state(rng0)
                            self._slots = None
                            return self.run(batches, extras, post)
                        self._recapture_forwards(extra_of(i), dev)
                        self._pkey = self._params.key()
                sl = self._slots[s].halves[h]
                main = mains[(i - first) % len(mains)]
                with torch.cuda.stream(main):
                    main.wait_event(ev_fps[s])
                    if ev_head[bs] is not None:  # the batch slot's last head is done with the pool
                        main.wait_event(ev_head[bs])
                    for d, e in zip(sl.extra, extra_of(i)):
                        d.copy_(e, non_blocking=True)
                    mark(i - first, "sa0", main)
                    sl.sa.replay()
                    ev_sa = main.record_event()
                    mark(i - first, "sa1", main)
                # the last `drain` batches run their heads on their own (by then idle)
                # compute streams: the tail stream runs ~2 heads behind the sa graphs, and at
                # the end of a run that backlog is the drain
                # consecutive batches' heads alternate between the tail streams
                ts = tails[(i - first) % len(tails)] if (sl.head is not None and self.head_on_tail and
                                                         i < len(batches) - drain) else main
                with torch.cuda.stream(ts):
                    if sl.head is not None:
                        if ts is not main:
                            ts.wait_event(ev_sa)
                        mark(i - first, "hd0", ts)
                        sl.head.replay()
                    out = _clone(sl.out)
                    # recorded before `post` (e.g. an all_gather) so the group's next fps
                    # replay does not wait for the collective; a later batch of the group
                    # replaces it (same streams, later in their order)
                    ev_read[s].append(ts.record_event() if sl.tail_reads_geometry else ev_sa)
                    if post is not None and ts is tail:
                        out = post(i, out)
                    ev_head[bs] = ts.record_event()
                    mark(i - first, "hd1", ts)
                if post is not None and ts is not tail:
                    # heads on a compute stream or on the second tail stream: `post` (e.g. the
                    # logits' all_gather, or BatchedGather's stack of earlier batches' outputs)
                    # still runs on one stream in batch order, so every rank's collectives
                    # execute in the order they were issued and a bundle's outputs are all
                    # complete on the stream that reads them
                    tail.wait_stream(ts)
                    with torch.cuda.stream(tail):
                        for t in _flat_tensors(out):
                            t.record_stream(tail)
                        out = post(i, out)
                outs.append(out)
                top_up(-1, (g if h == gb - 1 else g - 1) + ng)
        for g in geos[1:]:
            geo.wait_stream(g)
        self._pinned_evs[self._pinned_cur] = geo.record_event()  # uploads read it
        for st in [geo] + mains + tails:
            caller.wait_stream(st)
        return outs

    def _run_fused(self, batches, extra_of, post, first, outs, ngr, geos, mains, tails, tail,
                   ev_fps, ev_read, ev_head, top_up, check_params, dev, mark):
        """run()'s issue loop with fused group forwards: per geometry group one sa graph (on
        the compute streams in turn) and one head graph (tail stream) over its gb batches; the
        outputs are split into per-batch rows, `post` runs per batch in batch order."""
        gb, ng = self.gb, self.ngroups
        drain = int(tuning.get("drain_heads"))
        drain_groups = (drain + gb - 1) // gb
        for g in range(ngr):
            s = g % ng
            i0 = first + g * gb
            js = [i0 + h for h in range(gb) if i0 + h < len(batches)]
            top_up(g, -1)
            if check_params:  # (first group: its geometry is issued)
                check_params = False
                if self._params.key() != self._pkey:
                    if [id(m) for m in self._find_sas()] != [id(m) for m in self.sas]:
                        raise _Restart()
                    self._recapture_forwards(extra_of(i0), dev)
                    self._pkey = self._params.key()
            grp = self._slots[s]
            sl = grp.halves[0]
            B = grp.B
            main = mains[g % len(mains)]
            with torch.cuda.stream(main):
                main.wait_event(ev_fps[s])
                if ev_head[s] is not None:  # the slot's last head is done with the pool
                    main.wait_event(ev_head[s])
                for h in range(gb):
                    for d, e in zip(sl.extra, extra_of(js[h] if h < len(js) else js[0])):
                        d[h * B:(h + 1) * B].copy_(e, non_blocking=True)
                mark(i0 - first, "sa0", main)
                sl.sa.replay()
                ev_sa = main.record_event()
                mark(i0 - first, "sa1", main)
            ts = tails[g % len(tails)] if (sl.head is not None and self.head_on_tail and
                                           g < ngr - drain_groups) else main
            with torch.cuda.stream(ts):
                if sl.head is not None:
                    if ts is not main:
                        ts.wait_event(ev_sa)
                    mark(i0 - first, "hd0", ts)
                    sl.head.replay()
                full = _clone(sl.out)
                ev_read[s].append(ts.record_event() if sl.tail_reads_geometry else ev_sa)
                outs_g = [_rows(full, h * B, (h + 1) * B) for h in range(len(js))]
                if post is not None and ts is tail:
                    outs_g = [post(j, o) for j, o in zip(js, outs_g)]
                ev_head[s] = ts.record_event()
                mark(i0 - first, "hd1", ts)
            if post is not None and ts is not tail:
                tail.wait_stream(ts)
                with torch.cuda.stream(tail):
                    for t in _flat_tensors(full):
                        t.record_stream(tail)
                    outs_g = [post(j, o) for j, o in zip(js, outs_g)]
            outs.extend(outs_g)
            top_up(-1, g + ng)

    def _draw_all(self, k):
        """The pinned host buffer that receives the start draws of the next k groups, one row
        per group (one asynchronous upload per group, no per-draw pinning on the issue path).
        Rows are drawn by ``_draw_row`` just before their group's upload is issued -- batch by
        batch, each in layer order: the order k eager forwards take them -- so the host draws
        overlap the GPU work of earlier groups instead of delaying the first launch.  Two
        buffers alternate across calls; one is reused once the uploads of the call before last
        ran."""
        width = self.gb * sum(B for B, _ in self._draws)
        if not hasattr(self, "_pinned"):
            self._pinned, self._pinned_evs, self._pinned_cur = [None, None], [None, None], 0
        c = self._pinned_cur = 1 - self._pinned_cur
        if self._pinned_evs[c] is not None:
            self._pinned_evs[c].synchronize()
        buf = self._pinned[c]
        if buf is None or buf.shape[0] < k or buf.shape[1] != width:
            # both buffers at once: a page-locked allocation costs a host-side driver call
            # (hundreds of us), and the second buffer's would otherwise land inside the call
            # after the first -- in a benchmark, inside the first timed run
            rows = max(k, 64, *(b.shape[0] for b in self._pinned if b is not None and b.shape[1] == width))
            self._pinned = [torch.empty(rows, width, dtype=torch.long, pin_memory=True) for _ in range(2)]
            self._pinned_evs = [None, None]
            buf = self._pinned[c]
        return buf

    def _draw_row(self, buf, g, nh):
        """Group g's starts: batches 0..nh-1 of the group draw (in batch, then layer order) into
        their places of the start layout (see _capture); the empty places get 0."""
        gb = self.gb
        for h in range(gb):
            off = 0
            for B, N in self._draws:
                dst = buf[g, off + h * B:off + (h + 1) * B]
                if h < nh:
                    shard.draw_start_into(dst, N)
                else:
                    dst.zero_()
                off += gb * B
        return buf[g]
