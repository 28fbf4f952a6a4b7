"""Host-side logic on CPU: drop-in API surface, state_dict compatibility with the reference's
checkpoints, RNG parity of the sharded FPS draws, and the world_size-2 gloo data-parallel path."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import cases
from conftest import PKG, golden_names, load_golden

REF = "/root/reference/model"


def test_public_names_and_signatures():
    import inspect
    import pointnet2_utils as P  # the shim
    import pn2
    assert P.PointNetSetAbstraction is pn2.PointNetSetAbstraction
    sig = {
        "square_distance": ["src", "dst"],
        "index_points": ["points", "idx"],
        "farthest_point_sample": ["points", "number"],
        "query_ball_point": ["radius", "number", "points", "new_points"],
        "sample_and_group": ["points", "feature", "point_number", "sample_number", "radius", "returnfps"],
        "sample_and_group_all": ["points", "feature"],
    }
    for name, params in sig.items():
        assert list(inspect.signature(getattr(P, name)).parameters) == params
    assert list(inspect.signature(P.PointNetSetAbstraction.__init__).parameters)[1:] == [
        "point_number", "sample_number", "radius", "in_channel", "mlp", "group_all"]
    assert list(inspect.signature(P.PointNetSetAbstractionMsg.__init__).parameters)[1:] == [
        "point_number", "sample_number_list", "radius_list", "in_channel", "mlp_list", "num_category"]


@pytest.mark.parametrize("name", golden_names("head_"))
def test_heads_rebuild_reference_weights(name):
    """pn2.heads consume the RNG exactly like the reference heads: same seeded state_dict
    (hash recorded from the reference in the golden)."""
    from pn2 import heads as H
    head, B, N, kind, wseed, fseed = cases.HEAD_CASES[name]
    model = cases.build_head(H.HEADS[head], wseed)
    assert cases.state_hash(model) == str(load_golden("head_%s.npz" % name)["state_hash"])


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not present")
@pytest.mark.parametrize("head", ["pointnet2_cls_ssg", "pointnet2_cls_msg", "rotation_ssg",
                                  "translation_ssg", "rotation_msg", "translation_msg", "sign_ssg",
                                  "sign_msg"])
def test_reference_heads_import_drop_in_unchanged(head, monkeypatch):
    """The reference's own head files, imported with `pointnet2_utils` resolving to the
    drop-in, build, load a reference-built checkpoint (state_dict) strictly, and refuse CPU
    execution loudly instead of silently falling back."""
    import importlib
    import pn2.pointnet2_utils as ours
    monkeypatch.setattr(sys, "dont_write_bytecode", True)
    # the reference's own modules, for a checkpoint made by the real implementation
    monkeypatch.syspath_prepend(REF)
    for m in ("pointnet2_utils", head):
        sys.modules.pop(m, None)
    ref_mod = importlib.import_module(head)
    ref_sd = ref_mod.get_model().state_dict()
    sys.modules.pop(head, None)
    monkeypatch.setitem(sys.modules, "pointnet2_utils", ours)
    mod = importlib.import_module(head)
    assert mod.PointNetSetAbstraction is ours.PointNetSetAbstraction
    model = mod.get_model()
    model.load_state_dict(ref_sd, strict=True)
    sys.modules.pop(head, None)
    model.eval()
    x = torch.rand(2, 10 if "cls" not in head else 3, 64)
    args = (x, torch.rand(2, 3)) if head.startswith("translation") else (x,)
    with pytest.raises(RuntimeError, match="ROCm device tensors only"):
        with torch.no_grad():
            model(*args)


def test_sharded_draws_match_unsharded():
    from pn2 import shard
    torch.manual_seed(3)
    full = [shard.draw_start(64, 1024), shard.draw_start(64, 512)]
    parts = []
    for r in range(8):
        lo, hi = shard.shard_range(64, r, 8)
        torch.manual_seed(3)
        with shard.batch_shard(64, lo):
            parts.append((shard.draw_start(hi - lo, 1024), shard.draw_start(hi - lo, 512)))
    for layer in range(2):
        np.testing.assert_array_equal(torch.cat([p[layer] for p in parts]).numpy(), full[layer].numpy())
    assert shard.shard_range(10, 0, 4) == (0, 3) and shard.shard_range(10, 3, 4) == (8, 10)


def _gloo_worker(rank, world, port, out, B=8):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, PKG)
    from pn2 import shard
    lo, hi = shard.shard_range(B, rank, world)
    torch.manual_seed(21)
    with shard.batch_shard(B, lo):
        starts = shard.draw_start(hi - lo, 100)
        local = torch.stack([starts.double(), torch.full((hi - lo,), float(rank), dtype=torch.float64)], 1)
        got_spec = shard.all_gather_rows(local, sizes="shard")  # row counts from batch_shard
        # a tensor that is not per-cloud (one summary row per rank) inside batch_shard: the
        # default gathers the row counts
        summ = shard.all_gather_rows(torch.full((1, 2), float(rank), dtype=torch.float64))
        assert summ[:, 0].tolist() == [float(r) for r in range(world)]
    got = shard.all_gather_rows(local)  # row counts gathered from the ranks
    got_sizes = shard.all_gather_rows(local, sizes=shard.shard_sizes(B, world))
    if rank == 0:
        out.put((got.numpy(), got_spec.numpy(), got_sizes.numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("B,world", [(8, 2), (7, 2), (7, 3)])
def test_gloo_all_gather_and_rng_parity(B, world):
    """world_size 2-3 over gloo: every rank draws the full batch's FPS starts and keeps its
    shard; the gathered rows are the unsharded draw, in rank order -- also for uneven shards
    (B % world != 0), whether the row counts come from batch_shard, an explicit list, or a
    gather of the counts."""
    import random
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = random.randint(20000, 40000)
    procs = [ctx.Process(target=_gloo_worker, args=(r, world, port, q, B)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    torch.manual_seed(21)
    want = torch.randint(0, 100, (B,), dtype=torch.long).numpy()
    owner = np.concatenate([np.full(hi - lo, r) for r, (lo, hi) in
                            enumerate(shard_ranges(B, world))])
    for got in res:
        assert got.shape == (B, 2)
        np.testing.assert_array_equal(got[:, 0].astype(np.int64), want)
        np.testing.assert_array_equal(got[:, 1], owner)


def _batched_gather_worker(rank, world, port, out, B, every):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, PKG)
    from pn2 import shard
    lo, hi = shard.shard_range(B, rank, world)
    nb = 5
    # per batch i: two "heads" of different widths, rows tagged by cloud and batch
    outs = [[torch.arange(lo, hi, dtype=torch.float64)[:, None] * 10 + i + torch.zeros(1, 3, dtype=torch.float64),
             torch.full((hi - lo, 2), float(rank * 100 + i), dtype=torch.float64)] for i in range(nb)]
    with shard.batch_shard(B, lo):
        bg = shard.BatchedGather(every, total=nb)
        for i, o in enumerate(outs):
            bg(i, o)
        want = [[shard.all_gather_rows(h, sizes="shard") for h in o] for o in outs]
    if rank == 0:
        out.put(([[h.numpy() for h in r] for r in bg.results], [[h.numpy() for h in r] for r in want]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("B,world,every", [(8, 2, 2), (7, 3, 4), (7, 2, 1)])
def test_batched_gather_matches_per_batch(B, world, every):
    """shard.BatchedGather (the pipelined bench's exchange: one collective per `every` batches)
    returns, per batch, exactly what a per-batch all_gather_rows returns -- uneven shards, two
    heads, and a last partial bundle (5 batches)."""
    import random
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = random.randint(20000, 40000)
    procs = [ctx.Process(target=_batched_gather_worker, args=(r, world, port, q, B, every))
             for r in range(world)]
    for p in procs:
        p.start()
    got, want = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(got) == len(want) == 5
    for g, w in zip(got, want):
        for gh, wh in zip(g, w):
            np.testing.assert_array_equal(gh, wh)


BENCH = os.path.join(os.path.dirname(PKG), "bench.py")


@pytest.mark.parametrize("config,gpus", [("ssg", 2), ("pose", 3), ("pose", 8)])
def test_bench_launcher_plumbing(config, gpus):
    """`bench.py --gpus N` (no torchrun) starts N ranks itself with the torchrun environment;
    --plumbing-check runs their gloo group, shard split and uneven all_gather on the CPU (pose:
    the global B=64 over 3 ranks is uneven).  The JSON line must report n_gpus == N."""
    import json
    import subprocess
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(gpus), "--config", config,
                        "--plumbing-check"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["plumbing_check"] is True
    assert line["n_gpus"] == gpus
    assert line["global_batch"] == (64 if config == "pose" else 32 * gpus)


def test_bench_rejects_world_mismatch():
    """Under a launcher, --gpus must equal WORLD_SIZE (no silent one-rank run)."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--plumbing-check"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_count_gpus_without_hip(monkeypatch, tmp_path):
    """The launcher's parent counts GPUs from the KFD topology and the visibility variables,
    never through HIP (a parent that initialised HIP before forking its ranks is the hazard)."""
    sys.path.insert(0, os.path.dirname(PKG))
    import bench
    topo = tmp_path / "nodes"
    for i, simds in enumerate([0, 256, 256, 256]):  # node 0: the CPU
        d = topo / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text("cpu_cores_count 0\nsimd_count %d\n" % simds)
    for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    assert bench.count_gpus(str(topo)) == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1")
    assert bench.count_gpus(str(topo)) == 2
    assert bench.count_gpus(str(tmp_path / "absent")) == 0


def shard_ranges(B, world):
    sys.path.insert(0, PKG)
    from pn2 import shard
    return [shard.shard_range(B, r, world) for r in range(world)]
