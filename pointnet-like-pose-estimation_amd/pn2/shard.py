"""Batch sharding across GPUs (one process per GPU, RCCL over xGMI).

Every cloud of an eval-mode PointNet++ forward is independent (BatchNorm uses running stats,
FPS / ball query / grouping are per cloud), so a global batch splits into contiguous per-rank
shards with no exchange inside the forward.  Two things keep the sharded run identical to the
single-GPU run of the whole batch:

  * FPS start indices.  The reference draws ``torch.randint(0, N, (B,))`` from the CPU default
    generator once per SA layer (pointnet2_utils.py:59).  Inside ``batch_shard(global_B,
    offset)`` every rank draws the FULL-batch vector (same seed -> same stream on every rank)
    and keeps its slice, so the RNG stream advances exactly as in the unsharded run.
  * The only collective: ``all_gather_rows`` of the per-rank head outputs (logits, [B/W, k]
    fp32 -- a few hundred bytes, latency-bound over xGMI).
"""
import contextlib
import threading

import torch
import torch.distributed as dist

from . import tuning

_state = threading.local()


@contextlib.contextmanager
def batch_shard(global_batch, offset):
    """Within this context FPS start draws are taken for `global_batch` clouds and sliced at
    `offset` (this rank's first cloud)."""
    prev = getattr(_state, "spec", None)
    _state.spec = (int(global_batch), int(offset))
    try:
        yield
    finally:
        _state.spec = prev


@contextlib.contextmanager
def thread_generator(generator):
    """Within this context (this host thread) the FPS start draws come from `generator` (a CPU
    torch.Generator) instead of the CPU default generator.  The reference draws from the
    default generator (pointnet2_utils.py:59), so forwards running concurrently on several
    threads (mutilthreading/predict_test.py:44-63) interleave their draws in whatever order
    the threads happen to run; a generator per thread makes each thread's draws -- and its
    outputs -- reproducible.  None: the default generator."""
    prev = getattr(_state, "gen", None)
    _state.gen = generator
    try:
        yield
    finally:
        _state.gen = prev


def rng_state():
    """The state of the generator the start draws come from (this thread's thread_generator, or
    the CPU default generator) -- for a caller that must take draws back (set_rng_state)."""
    gen = getattr(_state, "gen", None)
    return gen.get_state() if gen is not None else torch.get_rng_state()


def set_rng_state(state):
    gen = getattr(_state, "gen", None)
    if gen is not None:
        gen.set_state(state)
    else:
        torch.set_rng_state(state)


def draw_start(B, N, pin=True):
    """CPU int64 [B]: the reference's randint draw (or this shard's slice of it), pinned (unless
    pin=False) so the host->device copy is asynchronous."""
    spec = getattr(_state, "spec", None)
    gen = getattr(_state, "gen", None)
    if spec is None:
        t = torch.randint(0, N, (B,), dtype=torch.long, generator=gen)
    else:
        gb, off = spec
        if off + B > gb:
            raise ValueError("batch_shard: shard [%d, %d) outside global batch %d" % (off, off + B, gb))
        t = torch.randint(0, N, (gb,), dtype=torch.long, generator=gen)[off:off + B]
    return t.pin_memory() if pin and torch.cuda.is_available() else t


def draw_start_into(dst, N):
    """draw_start(len(dst), N) written into the CPU int64 vector dst: the same draw (the same
    generator consumption and values), straight into dst when this process draws the whole
    batch -- the pipeline's pinned start rows, without a temporary and a copy per draw."""
    spec = getattr(_state, "spec", None)
    B = dst.shape[0]
    if spec is None or (spec[0] == B and spec[1] == 0):
        torch.randint(0, N, (B,), dtype=torch.long, out=dst, generator=getattr(_state, "gen", None))
    else:
        dst.copy_(draw_start(B, N, pin=False))


def device_start(B, N, device):
    """The FPS start draw as a device tensor.  Inside a graph capture (graphs.GraphedForward)
    the draw is not taken here: the capture reads a static device slot that every replay
    refills with a fresh draw, taken in the same order as the eager forward takes them."""
    rec = getattr(_state, "graph", None)
    if rec is not None:
        return rec(B, N, device)
    return draw_start(B, N).to(device, non_blocking=True)


def recording():
    """Whether a graph record/capture's start source is installed (start_source)."""
    return getattr(_state, "graph", None) is not None


def host_start(B, N, device):
    """The FPS start draw as the eager forward hands it to pn2_fps_host_ws_f32: a CPU int64
    tensor (the launch carries the values in its kernel arguments -- no host->device copy), or,
    inside a graph record/capture, what the installed start source returns (device_start)."""
    rec = getattr(_state, "graph", None)
    if rec is not None:
        return rec(B, N, device)
    return draw_start(B, N, pin=False)


@contextlib.contextmanager
def start_source(fn):
    """Route device_start(B, N, device) to fn for the duration (graph record/capture)."""
    prev = getattr(_state, "graph", None)
    _state.graph = fn
    try:
        yield
    finally:
        _state.graph = prev


def shard_range(global_batch, rank, world):
    """Contiguous [lo, hi) of clouds owned by `rank` (the remainder goes to the first ranks)."""
    base, rem = divmod(global_batch, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def shard_sizes(global_batch, world):
    """Clouds owned by every rank, in rank order (``shard_range``'s split)."""
    return [hi - lo for lo, hi in (shard_range(global_batch, r, world) for r in range(world))]


def all_gather_rows(local, group=None, sizes=None):
    """Concatenate every rank's [b_r, ...] tensor along dim 0, in rank order (RCCL all_gather on
    GPU tensors, gloo on CPU ones).

    Shards may be uneven (``shard_range`` gives the remainder to the first ranks).  The row
    counts come from `sizes`: a list, or ``"shard"`` -- every rank's ``shard_range`` of the
    enclosing ``batch_shard``'s global batch (for per-cloud tensors of the shard, e.g. the
    logits: no extra collective) -- or, by default, from one extra all_gather of the counts
    (any row counts).  The choice must be the same on every rank (it decides which collectives
    run).  Every rank's rows are padded to the largest count for the one fixed-size collective
    and trimmed after it."""
    if not dist.is_available() or not dist.is_initialized():
        return local
    world = dist.get_world_size(group)
    if world == 1 and not tuning.get("force_gather"):
        return local
    local = local.contiguous()
    if isinstance(sizes, str):
        if sizes != "shard":
            raise ValueError("all_gather_rows: sizes must be a list, 'shard' or None")
        spec = getattr(_state, "spec", None)
        if spec is None:
            raise ValueError("all_gather_rows(sizes='shard') outside batch_shard")
        sizes = shard_sizes(spec[0], world)
        if sizes[dist.get_rank(group)] != local.shape[0]:
            raise ValueError("all_gather_rows: %d rows on rank %d, batch_shard(%d) gives %d"
                             % (local.shape[0], dist.get_rank(group), spec[0],
                                sizes[dist.get_rank(group)]))
    if sizes is None:
        n = torch.tensor([local.shape[0]], dtype=torch.long, device=local.device)
        ns = torch.empty(world, dtype=torch.long, device=local.device)
        dist.all_gather_into_tensor(ns, n, group=group)
        sizes = [int(v) for v in ns.tolist()]
    sizes = [int(v) for v in sizes]
    if len(sizes) != world:
        raise ValueError("all_gather_rows: %d sizes for %d ranks" % (len(sizes), world))
    rest = tuple(local.shape[1:])
    m = max(sizes)
    if m != local.shape[0]:
        pad = local.new_zeros((m,) + rest)
        pad[:local.shape[0]] = local
        local = pad
    out = torch.empty((world * m,) + rest, dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, local, group=group)
    if all(n == m for n in sizes):
        return out
    return torch.cat([out[r * m:r * m + n] for r, n in enumerate(sizes)])


class BatchedGather:
    """A pipeline ``post`` callback that gathers the heads' per-batch outputs across the ranks
    in one collective per `every` batches instead of one per batch: the outputs of the batches
    since the last gather are stacked along a new dim 1 ([b_r, n, ...] per head), all-gathered
    by rows (``all_gather_rows``) and split back, so ``results`` holds, per batch, exactly what
    a per-batch ``all_gather_rows`` returns.  Every rank must see the same call sequence.
    `total` (the batch count) flushes the last partial bundle; ``flush()`` does it otherwise.
    (One RCCL collective per batch costs ~10 % of the pipelined SSG rate even on one GPU --
    DESIGN.md §6; batching the exchange keeps the queues to the pipeline's own.)"""

    def __init__(self, every, total=None, sizes="shard"):
        self.every, self.total, self.sizes = max(1, int(every)), total, sizes
        self.pending, self.results, self.calls = [], [], 0

    def __call__(self, i, out):
        heads = list(out) if isinstance(out, (tuple, list)) else [out]
        self.pending.append(heads)
        self.calls += 1
        if len(self.pending) == self.every or (self.total is not None and self.calls == self.total):
            self.flush()
        return out

    def flush(self):
        if not self.pending:
            return
        n = len(self.pending)
        per_head = []
        for h in range(len(self.pending[0])):
            local = torch.stack([p[h] for p in self.pending], 1)
            g = all_gather_rows(local, sizes=self.sizes)
            per_head.append([g[:, j] for j in range(n)])
        for j in range(n):
            hs = [ph[j] for ph in per_head]
            self.results.append(hs if len(hs) > 1 else hs[0])
        self.pending = []
