"""The multi-GPU product path's collective on the RCCL backend, at world size 1 (the box has one
GPU; the N-rank path is covered on gloo in test_host.py).

bench.py's pipelined run gathers every head's logits across the ranks from the pipeline's `post`
hook, through shard.BatchedGather -> shard.all_gather_rows -> torch.distributed's "nccl" backend
(RCCL).  With tuning force_gather=1 the collective runs even in a 1-rank group, so the RCCL
all_gather sits on the pipeline's tail stream exactly as in an 8-GPU run: the gathered,
pipelined logits must equal the eager logits bit for bit -- with one tail stream, and with
tail_streams=2 (heads of consecutive batches alternating between two tail streams; `post`
still runs on one stream in batch order)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

import cases

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def rccl_group():
    assert torch.cuda.is_available()
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    assert not dist.is_initialized()
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _free_port(), rank=0,
                            world_size=1, device_id=torch.device(DEV, 0))
    assert dist.get_backend() == "nccl"
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("tail_streams,compute_streams", [(1, 2), (2, 1)])
@pytest.mark.parametrize("every", [1, 3])
def test_pipelined_rccl_gather_equals_eager(rccl_group, tail_streams, compute_streams, every):
    from pn2 import heads as H
    from pn2 import shard, tuning
    from pn2.pipeline import GraphedPipeline
    model = cases.build_head(H.HEADS["pointnet2_cls_ssg"], 1500).to(DEV)
    B, N, n = 32, 1024, 7
    xs = [cases.cloud("uniform3", B, N, 1600 + i).permute(0, 2, 1).contiguous().to(DEV) for i in range(n)]
    torch.manual_seed(21)
    with torch.no_grad():
        eager = [model(x)[0] for x in xs]
    with tuning.override(force_gather=1, tail_streams=tail_streams):
        gp = GraphedPipeline(model, compute_streams=compute_streams)
        assert gp.tail_streams == tail_streams
        bg = shard.BatchedGather(every, total=n)
        torch.manual_seed(21)
        with shard.batch_shard(B, 0):
            gp.run(xs, post=lambda i, o: bg(i, o[0]))
        torch.cuda.synchronize()
    assert len(bg.results) == n
    for i in range(n):
        np.testing.assert_array_equal(bg.results[i].cpu().numpy(), eager[i].cpu().numpy(),
                                      err_msg="batch %d" % i)


def test_all_gather_rows_rccl_uneven_sizes(rccl_group):
    """all_gather_rows over RCCL with explicit sizes and the count exchange (sizes=None)."""
    from pn2 import shard, tuning
    x = torch.randn(5, 7, device=DEV)
    with tuning.override(force_gather=1):
        a = shard.all_gather_rows(x)
        b = shard.all_gather_rows(x, sizes=[5])
    torch.testing.assert_close(a, x, rtol=0, atol=0)
    torch.testing.assert_close(b, x, rtol=0, atol=0)
