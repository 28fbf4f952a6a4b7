"""GPU parity of the heads' fused eval FC tail (pn2_fc_tail_f32: fc1 + bn1 + ReLU, fc2 + bn2 +
ReLU, fc3, and the classifiers' log_softmax + argmax -- pointnet2_cls_ssg.py:31-38) against the
reference's modules in float64, row-count invariance (sharded batches stay bit-identical), and
group_all's new_points zeros filled by the MLP launch."""
import numpy as np
import pytest
import torch

import cases

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(head, seed):
    from pn2 import heads as H
    torch.manual_seed(seed)
    m = getattr(H, head)()
    cases.randomize_bn(m, seed)
    return m.eval()


def _ref_tail(m, x):
    """The reference's tail (eval: dropout = identity) in float64 on the CPU."""
    md = {k: v.detach().double().cpu() for k, v in m.state_dict().items()}

    def bn(y, p):
        return (y - md[p + ".running_mean"]) / torch.sqrt(md[p + ".running_var"] + 1e-5) * \
            md[p + ".weight"] + md[p + ".bias"]
    y = x.double().cpu()
    y = torch.relu(bn(y @ md["fc1.weight"].T + md["fc1.bias"], "bn1"))
    y = torch.relu(bn(y @ md["fc2.weight"].T + md["fc2.bias"], "bn2"))
    return y @ md["fc3.weight"].T + md["fc3.bias"]


@pytest.mark.parametrize("B", [1, 5, 20, 32, 64])
@pytest.mark.parametrize("head", ["ClsSSG", "RotationSSG", "SignSSG"])
def test_fc_tail_matches_reference(head, B):
    m = _model(head, 11).to(DEV)
    x = torch.relu(torch.randn(B, 1024, generator=torch.Generator().manual_seed(B))).to(DEV)
    ref = _ref_tail(m, x)
    with torch.no_grad():
        if head.startswith("Cls"):
            got, pred = m._fc_log_softmax(x)
            want = torch.log_softmax(ref, -1)
            np.testing.assert_array_equal(pred.cpu().numpy(), got.cpu().double().argmax(1).numpy())
            top2 = torch.topk(want, 2, dim=1).values
            sure = (top2[:, 0] - top2[:, 1]) > 1e-4
            np.testing.assert_array_equal(pred.cpu().numpy()[sure.numpy()], want.argmax(1).numpy()[sure.numpy()])
        else:
            got = m._fc(x)
            want = ref
    np.testing.assert_allclose(got.cpu().double().numpy(), want.numpy(), rtol=1e-5,
                               atol=1e-5 * float(want.abs().max()))


def test_fc_tail_rows_independent_of_batch():
    """Every output row is computed the same way whatever the row count: a shard of the batch
    gives the bits of the whole batch's rows (the data-parallel path relies on it)."""
    m = _model("ClsSSG", 4).to(DEV)
    x = torch.relu(torch.randn(64, 1024, generator=torch.Generator().manual_seed(0))).to(DEV)
    with torch.no_grad():
        full, pf = m._fc_log_softmax(x)
        for lo, hi in ((0, 8), (8, 19), (19, 64)):
            part, pp = m._fc_log_softmax(x[lo:hi])
            np.testing.assert_array_equal(part.cpu().numpy(), full[lo:hi].cpu().numpy())
            np.testing.assert_array_equal(pp.cpu().numpy(), pf[lo:hi].cpu().numpy())


def test_fc_tail_repeated_calls_same_bits():
    """Back-to-back calls on one stream and a graph replay give the same bits."""
    m = _model("ClsSSG", 6).to(DEV)
    x = torch.relu(torch.randn(32, 1024, generator=torch.Generator().manual_seed(1))).to(DEV)
    with torch.no_grad():
        outs = [m._fc_log_softmax(x)[0].cpu().numpy() for _ in range(5)]
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            m._fc_log_softmax(x)  # warm-up on the capture stream
            torch.cuda.synchronize()
            g.capture_begin()
            gy, _ = m._fc_log_softmax(x)
            g.capture_end()
        torch.cuda.current_stream().wait_stream(s)
        for _ in range(3):
            g.replay()
            torch.cuda.synchronize()
            outs.append(gy.cpu().numpy())
    for o in outs[1:]:
        np.testing.assert_array_equal(o, outs[0])


def test_group_all_new_points_zero_filled():
    """group_all's new_points are the reference's zeros (pointnet2_utils.py:136), written by the
    MLP's last launch into a fresh (uninitialised) tensor."""
    import pn2
    torch.manual_seed(2)
    sa = pn2.PointNetSetAbstraction(None, None, None, 259, [256, 512, 1024], True).to(DEV).eval()
    pts = torch.rand(8, 3, 128, device=DEV)
    feat = torch.rand(8, 256, 128, device=DEV)
    junk = torch.full((1 << 16,), float("nan"), device=DEV)  # poison the caching allocator
    del junk
    with torch.no_grad():
        newp, _ = sa(pts, feat)
    assert newp.shape == (8, 3, 1)
    assert torch.equal(newp, torch.zeros_like(newp))


def test_fc_tail_argmax_first_of_ties():
    """Equal logits: the first index wins (x.data.max(1)[1] on the reference's CPU tensors), also
    when the tie spans the wave's lanes (40 classes, one per lane)."""
    from pn2 import heads as H
    torch.manual_seed(8)
    m = H.ClsSSG(num_category=40)
    cases.randomize_bn(m, 8)
    m.eval()
    with torch.no_grad():
        m.fc3.weight.zero_()
        m.fc3.bias.zero_()
        m.fc3.bias[[7, 13, 30]] = 1.0
    m = m.to(DEV)
    with torch.no_grad():
        x = torch.relu(torch.randn(6, 1024, generator=torch.Generator().manual_seed(3))).to(DEV)
        logp, pred = m._fc_log_softmax(x)
    assert pred.tolist() == [7] * 6
    want = torch.log_softmax(m.fc3.bias.detach().double().cpu(), 0)
    np.testing.assert_allclose(logp.cpu().double().numpy(), want.expand(6, -1).numpy(), rtol=1e-6, atol=1e-6)
