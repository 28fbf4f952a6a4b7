"""Host-side helpers of the graphed paths (CPU): the cached parameter-state key must change
whenever a captured graph would be stale, and the pipeline's in-place start draws must equal
the reference-order draws (values and generator consumption)."""
import torch

from pn2 import heads as H
from pn2 import shard
from pn2.graphs import ParamState, _module_tensors


def _full_key(m):
    return tuple((t.data_ptr(), t._version) for t in _module_tensors(m))


def test_param_state_tracks_in_place_and_assignment():
    m = H.ClsSSG().eval()
    ps = ParamState(m)
    k = ps.key()
    assert k == _full_key(m)
    assert ps.key() == k  # cached walk, unchanged state
    next(b for n, b in m.sa1.named_buffers() if n.endswith("running_mean")).add_(0.25)
    k2 = ps.key()
    assert k2 != k and k2 == _full_key(m)
    m.fc1.weight = torch.nn.Parameter(m.fc1.weight.detach().clone())  # re-assigned slot
    k3 = ps.key()
    assert k3 != k2 and k3 == _full_key(m)
    m.sa2.mlp_convs[0] = torch.nn.Conv2d(131, 128, 1)  # a replaced submodule
    k4 = ps.key()
    assert k4 != k3 and k4 == _full_key(m)
    m.fc1.register_buffer("extra", torch.zeros(3))  # a new entry
    assert ps.key() == _full_key(m) and len(ps.key()) == len(k4) + 1
    with torch.no_grad():
        m.fc2.weight.data = m.fc2.weight.data.clone()  # new storage, same object
    assert ps.key() == _full_key(m)


def test_draw_start_into_matches_draw_start():
    for spec in (None, (16, 0), (24, 8)):
        dst = torch.empty(16 if spec is None or spec[0] == 16 else 8, dtype=torch.long)
        B = dst.shape[0]
        ctx = shard.batch_shard(*spec) if spec else None

        def draws(into):
            torch.manual_seed(11)
            if into:
                shard.draw_start_into(dst, 1000)
                a = dst.clone()
            else:
                a = shard.draw_start(B, 1000, pin=False)
            return a, torch.randint(0, 1 << 30, (4,))  # the generator's state after the draw

        if ctx:
            with ctx:
                got, want = draws(True), draws(False)
        else:
            got, want = draws(True), draws(False)
        assert torch.equal(got[0], want[0]) and torch.equal(got[1], want[1])
