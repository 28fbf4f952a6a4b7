"""HIP-graph replay of an eval-mode forward (whole head: SA layers + FC head).

An eager PointNet++ forward is ~35 launches, most of them the head's small torch kernels; on
MI355X the host cannot issue them as fast as the GPU retires them, so the GPU idles between
forwards.  ``GraphedForward`` captures the forward once per input signature and replays it:
one launch per forward, identical kernels and numbers.

RNG parity.  The reference draws the FPS start indices from the CPU generator, one
``torch.randint(0, N, (B,))`` per SA layer in forward order (pointnet2_utils.py:59).  The first
call for a signature runs eagerly (that call's real result; it consumes its draws and records
their shapes); the capture that follows reads the start indices from static device slots and
consumes nothing.  Every replay takes the draws again -- same calls, same order, same
``shard.batch_shard`` slicing as eager -- uploads them into the slots and replays, so a mixed
sequence of eager and graphed forwards walks the CPU RNG stream exactly as all-eager would.

Outputs of a replay are the graph's static tensors: valid until the next call of the same
``GraphedForward`` (clone them to keep them).  A change of any parameter or buffer (data
pointer or in-place version), of the input signature, or of train/eval mode triggers a new
eager call + capture; training / autograd calls always run eagerly.
"""
import torch

from . import ops, shard


def _sig(args):
    return tuple((tuple(a.shape), tuple(a.stride()), a.dtype, a.device) for a in args)


def _module_tensors(model):
    """Every parameter and buffer of `model` (the same tensors as parameters() + buffers(),
    shared ones possibly twice): a direct walk of the module tree, ~6x cheaper on the host than
    the generator chain, which took 160-240 us for a PointNet++ head -- paid per replay call
    by the graph key below."""
    out = []

    def walk(m):
        out.extend(t for t in m._parameters.values() if t is not None)
        out.extend(t for t in m._buffers.values() if t is not None)
        for c in m._modules.values():
            if c is not None:
                walk(c)

    walk(model)
    return out


class ParamState:
    """(data_ptr, _version) of every parameter and buffer of a module tree -- what a captured
    graph bakes in -- with the tree walk cached.  The cache holds every slot of the tree (each
    ``_parameters`` / ``_buffers`` / ``_modules`` entry and the size of each of those dicts);
    it is re-walked only when a slot no longer holds the object it held or a dict changed size
    (an assignment, a new or deleted entry), which an identity check finds in a fraction of the
    walk's host time (~80 -> ~45 us for a PointNet++ head, before every pipelined run)."""

    def __init__(self, model):
        self.model = model
        self._slots = None
        self._sizes = None
        self._ts = None

    def _walk(self):
        slots, sizes, ts = [], [], []

        def walk(m):
            for d in (m._parameters, m._buffers, m._modules):
                sizes.append((d, len(d)))
                for k, v in d.items():
                    slots.append((d, k, v))
                    if v is not None:
                        if d is m._modules:
                            walk(v)
                        else:
                            ts.append(v)

        walk(self.model)
        self._slots, self._sizes, self._ts = slots, sizes, ts

    def key(self):
        if (self._slots is None or any(len(d) != n for d, n in self._sizes) or
                any(d.get(k) is not v for d, k, v in self._slots)):
            self._walk()
        return tuple((t.data_ptr(), t._version) for t in self._ts)


class GraphedForward:
    def __init__(self, model):
        self.model = model
        self._key = None
        self._graph = None
        self._params = None

    def _state_key(self, args):
        if self._params is None:
            self._params = ParamState(self.model)
        return (_sig(args), ops.current_precision()) + self._params.key()

    def _eager(self, args):
        draws = []

        def record(B, N, device):
            draws.append((B, N))
            return shard.draw_start(B, N).to(device, non_blocking=True)

        with torch.no_grad(), shard.start_source(record):
            out = self.model(*args)
        return out, draws

    def _capture(self, args, draws):
        dev = args[0].device
        self._static_in = [a.clone() for a in args]
        self._slots = [torch.zeros(B, dtype=torch.long, device=dev) for B, _ in draws]
        self._draws = draws
        it = iter(self._slots)

        def static_slot(B, N, device):
            return next(it)

        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize(dev)
        with torch.no_grad(), shard.start_source(static_slot), torch.cuda.graph(g):
            self._static_out = self.model(*self._static_in)
        self._graph = g

    def __call__(self, *args):
        if self.model.training or (torch.is_grad_enabled() and any(
                p.requires_grad for p in self.model.parameters())):
            return self.model(*args)
        key = self._state_key(args)
        if key != self._key or self._graph is None:
            out, draws = self._eager(args)
            self._graph = None
            self._capture(args, draws)
            self._key = self._state_key(args)  # capture allocations do not touch parameters
            return out
        for s, a in zip(self._static_in, args):
            s.copy_(a, non_blocking=True)
        for slot, (B, N) in zip(self._slots, self._draws):
            slot.copy_(shard.draw_start(B, N), non_blocking=True)
        self._graph.replay()
        return self._static_out
