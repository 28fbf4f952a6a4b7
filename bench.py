"""Throughput benchmark: point-clouds/sec of the pointnet2_cls_ssg forward (eval), B=32 clouds
of N=1024 points per GPU, on the MI355X-native SA path.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config ssg|msg|pose|stress|v1]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

One step = one forward of the head over every rank's batch shard (weak scaling: B clouds per
GPU, global batch = B*N) followed by the RCCL all_gather of the logits -- the only exchange the
data-parallel path has.  Inputs are resident in HBM before the timed region, which carries no
instrumentation.  Rank 0 prints one JSON line (contract in the task statement) with:
  value         clouds/s of K steps through pn2.pipeline.GraphedPipeline with EVERY LAUNCH ONE
                B-cloud BATCH (geometry_batches=1, fuse=False): independent B=32 forwards
                overlapped on streams -- each batch's geometry (FPS + ball queries) replayed from a
                HIP graph on one of two geometry streams, its SA forward on a compute stream, its
                head on a tail stream; every step computes exactly its eager forward, with the
                same CPU-RNG draws.  --no-pipeline times plain eager steps instead, --graph whole-
                forward HIP-graph replays.
  value_fused   the same K batches through a pipeline that fuses --fused-batches (4) consecutive
                batches into every launch (launch_batch = 4 x B): a serving mode, not the metric.
  eager_value   the same K steps one after the other, op by op (B / forward time).
  eager_value_reference_head
                the same, through pn2.heads.ReferenceForward: the reference head's forward
                restated call for call (pointnet2_cls_ssg.py:22-38), i.e. what the unchanged
                reference caller gets through the drop-in.
  roofline      dominant op = pn2_sa_mlp_max_f32 (gather + shared MLP + max; sa_chain_kernel /
                dense_*_kernel): achieved = algorithmic fp32 FLOPs (2*M*sum(cin*cout) per call,
                cin unpadded) / call duration timed with HIP events on the launch stream, over a
                further K eager steps (profiles/ has the rocprofv3 check).  The products are
                fp32-accurate splits on the 16-bit matrix cores (split fp16: 3 MFMAs per fp32
                product; split bf16: 6), so peak = the flops-weighted ceiling of the mix the calls
                ran, from the fp16/bf16 dense MFMA peak 2516.8 TFLOP/s (MI355X_MICROARCH.md).
                traffic = HBM bytes per call from rocprofv3 PMC (profiles/pmc_traffic.json).
  roofline_ball_query
                query_ball_point, the north star's named kernel: VALU-bound, HBM fraction beside.
  cpu_baseline  oracle/torch_ref.py -- the reference's formulation in torch-CPU ops -- timed on
                this host's cores on a bounded sample (rank 0, N=1 only).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "pointnet-like-pose-estimation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "point-clouds/sec forward, SSG B=32 N=1024, at 1/2/4/8 MI355X"
PEAK_F32_MFMA = 157.3  # TFLOP/s, MI355X_MICROARCH.md chip-level table (dense fp32 MFMA)
PEAK_BF16_MFMA = 16 * PEAK_F32_MFMA  # TFLOP/s, dense bf16 MFMA (2516.8)
PEAK_SPLIT = PEAK_BF16_MFMA / 6  # fp32-equivalent ceiling of 6-product split-bf16 MFMA
# fp32-equivalent ceiling of an MLP call by the planes per operand its kernels ran with
# (pn2_sa_mlp_last_planes): 3 = split bf16 (6 MFMAs per product), 2 = split fp16 (3; the fp16
# dense MFMA rate equals bf16's), 1 = bf16 (1), 0 = the fp32 MFMA kernels
PEAK_BY_PLANES = {3: PEAK_BF16_MFMA / 6, 2: PEAK_BF16_MFMA / 3, 1: PEAK_BF16_MFMA, 0: None}
PEAK_HBM = 8000.0      # GB/s
PEAK_F32_VALU = 157.3  # TFLOP/s, MI355X_MICROARCH.md (fp32 vector)

CONFIGS = {
    # name: (head, clouds per GPU, points, cloud kind, description)
    "ssg": ("pointnet2_cls_ssg", 32, 1024, "uniform3", "pointnet2_cls_ssg forward, B=32/GPU, N=1024"),
    "msg": ("pointnet2_cls_msg", 32, 4096, "uniform3", "pointnet2_cls_msg forward, B=32/GPU, N=4096"),
    # BASELINE config 4: B=64 batch-sharded across the GPUs (strong scaling: the global batch is
    # fixed, each rank runs its shard_range slice)
    "pose": ("rotation_ssg+translation_ssg", 64, 2048, "onehot10",
             "rotation_ssg + translation_ssg forward, global B=64 sharded over the GPUs, N=2048, 10-ch"),
    "stress": ("pointnet2_cls_ssg", 128, 16384, "uniform3", "pointnet2_cls_ssg forward, B=128/GPU, N=16384"),
    # BASELINE config 1 (the reference runs it on the CPU): PointNet-v1 on the v1 kernels
    "v1": ("pointnet_cls", 8, 1024, "uniform3", "pointnet_cls (PointNet v1) forward, B=8/GPU, N=1024"),
}
# configs whose batch is a fixed global batch split over the ranks; the others are B per GPU
STRONG = {"pose"}
# MLP arithmetic per config: BASELINE config 5 (stress) asks for features/MLP in bf16, the
# others are the reference's fp32
DEFAULT_PRECISION = {"stress": "bf16"}
# Geometry streams of the graphed pipeline.  At one batch per launch (the headline) each
# batch's FPS chain takes ~550-650 us of its stream under the compute kernels' contention
# (tools/debug/gpipe_events.py) against a ~270 us batch period, so four geometry streams, and
# the ball queries run in each batch's forward on the compute streams (SSG K = 20: 121-123k vs
# 96-110k with two streams and the queries on the geometry streams); with the geometry off the
# critical path the heads' tail stream backs up, so consecutive heads alternate between two tail
# streams (119.8-121.9k; 8 hardware queues: 4 geometry + 2 compute + 2 tail).  Fused launches
# (value_fused) keep r05's choice per config -- STRESS's N=16384 FPS needs two, the others one
# with a tail stream for the heads.
DEFAULT_GEOMETRY_STREAMS = {"stress": 2}
# batch slots of the graphed pipeline (at least 4 per geometry group)
DEFAULT_SLOTS = 16


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)  # pipelined: K batches in one pass, fill amortised
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="ssg", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bound on the CPU baseline sample")
    ap.add_argument("--no-kernel-timer", action="store_true")
    ap.add_argument("--no-settled", action="store_true",
                    help="skip the second pipelined measurement after an ~80 ms settle")
    ap.add_argument("--graph", action="store_true", help="replay the forward as a HIP graph")
    ap.add_argument("--eager-pipeline", action="store_true",
                    help="pipelined launch issued op by op (pn2.pipeline.PipelinedForward) "
                         "instead of replayed from HIP graphs (GraphedPipeline, the default)")
    ap.add_argument("--tail", action="store_true",
                    help="eager pipeline: run the head on its own stream (default off there)")
    ap.add_argument("--no-tail", action="store_true",
                    help="graphed pipeline: keep the head on the compute stream")
    ap.add_argument("--slots", type=int, default=None,
                    help="graphed pipeline: batch slots (a multiple of --geometry-batches; the "
                         "geometry runs slots/geometry-batches - 1 groups ahead; default 4 "
                         "groups)")
    ap.add_argument("--compute-streams", type=int, default=None,
                    help="graphed pipeline: consecutive batches' forwards alternate between this "
                         "many compute streams (1 or 2; default 2 with shared CUs)")
    ap.add_argument("--geometry-batches", type=int, default=1,
                    help="graphed pipeline: consecutive batches whose geometry (FPS + ball "
                         "queries) runs as one replay over their clouds side by side (default 1: "
                         "every launch of the headline value is one B-cloud batch)")
    ap.add_argument("--fuse", action="store_true",
                    help="graphed pipeline: one forward (sa + head graphs) per geometry group, "
                         "its batches side by side (launches of geometry-batches x B clouds)")
    ap.add_argument("--fused-batches", type=int, default=4,
                    help="after the headline, the same K batches through a pipeline that fuses "
                         "this many consecutive batches into every launch (value_fused, "
                         "launch_batch = this x B); 0 skips it")
    ap.add_argument("--no-reference-head", action="store_true",
                    help="skip eager_value_reference_head (the unchanged reference head's "
                         "forward through the drop-in, pn2.heads.ReferenceForward)")
    ap.add_argument("--geometry-streams", type=int, default=None,
                    help="graphed pipeline: 2 = consecutive groups' FPS chains on two streams "
                         "(default 2 for --config stress, else 1)")
    ap.add_argument("--geometry-bq", type=int, choices=(0, 1), default=None,
                    help="graphed pipeline: 1 = the ball queries on the geometry streams after each "
                         "FPS, 0 = in each batch's forward (default 0 at one batch per launch)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="plain eager steps (default for single-head configs: pn2.pipeline)")
    ap.add_argument("--precision", choices=("fp32", "bf16"), default=None,
                    help="shared-MLP arithmetic (default: bf16 for --config stress, else fp32)")
    ap.add_argument("--geometry-cus", type=int, default=0,
                    help="CUs reserved for the FPS chain (0: streams share every CU)")
    ap.add_argument("--hw-queues", type=int, default=8,
                    help="GPU_MAX_HW_QUEUES for this process (0: leave the environment's)")
    ap.add_argument("--gather-every", type=int, default=8,
                    help="pipelined runs: all_gather the head outputs of this many batches in "
                         "one collective (1: one collective per batch)")
    ap.add_argument("--force-rccl", action="store_true",
                    help="run the per-step all_gather of the head outputs through RCCL even on "
                         "one GPU (a 1-rank group): measures the collective's cost")
    ap.add_argument("--plumbing-check", action="store_true",
                    help="no GPU work: ranks join a gloo group, all_gather their shard ranges "
                         "and rank 0 prints a JSON line with n_gpus (tests the launcher on CPU)")
    return ap.parse_args()


def plumbing_check(a):
    """CPU check of the multi-rank plumbing: the process group, the shard split of the global
    batch and the uneven-shard all_gather -- the launch path a --gpus N run takes, minus the
    GPU."""
    from pn2 import shard
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    _, B, N, _, desc = CONFIGS[a.config]
    gB = B if a.config in STRONG else B * world
    lo, hi = shard.shard_range(gB, rank, world)
    rows = shard.all_gather_rows(torch.arange(lo, hi, dtype=torch.float64)[:, None])
    ok = rows[:, 0].tolist() == list(range(gB))
    if rank == 0:
        print(json.dumps({"plumbing_check": ok, "n_gpus": world, "global_batch": gB,
                          "rank_env": {k: os.environ.get(k) for k in
                                       ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR")},
                          "config": {"workload": desc, "parallelism": "dp%d" % world}}))
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


def build_models(cfg, dev):
    import cases
    from pn2 import heads
    head = CONFIGS[cfg][0]
    from pn2 import heads_v1
    names = head.split("+")
    models = []
    for i, n in enumerate(names):
        torch.manual_seed(1000 + i)
        m = heads.HEADS[n]() if n in heads.HEADS else heads_v1.HEADS_V1[n]()
        cases.randomize_bn(m, 2000 + i)
        models.append(m.eval().to(dev))
    return names, models


def make_inputs(cfg, B, lo, dev, rank, gB):
    import cases
    head, _, N, kind, _ = CONFIGS[cfg]
    if cfg in STRONG:  # this rank's slice [lo, lo + B) of one seeded global batch
        x = cases.cloud(kind, gB, N, 7)[lo:lo + B]
        mean = torch.randn(gB, 3, generator=torch.Generator().manual_seed(99))[lo:lo + B]
    else:  # B clouds per rank: a per-rank seed, same distribution
        x = cases.cloud(kind, B, N, 7 + rank)
        mean = torch.randn(B, 3, generator=torch.Generator().manual_seed(99 + rank))
    x = x.permute(0, 2, 1).contiguous().to(dev)  # [B, C, N] model input
    return x, mean.to(dev)


def step(names, models, x, mean, gB, lo):
    """One forward of every head over this rank's shard + the logits all_gather.  `models` are
    nn.Modules (eager) or pn2.graphs.GraphedForward wrappers."""
    from pn2 import shard
    outs = []
    with torch.no_grad(), shard.batch_shard(gB, lo):
        for n, m in zip(names, models):
            o = m(x, mean) if n.startswith("translation") else m(x)
            o = o[0] if isinstance(o, tuple) else o
            outs.append(shard.all_gather_rows(o, sizes="shard"))
    return outs


def cpu_baseline(seconds):
    """Reference formulation (oracle/torch_ref.py) on the host cores, bounded sample."""
    import cases
    from oracle import torch_ref
    from pn2 import heads
    # the GPU box shows every CPU of the host; our share is OMP_NUM_THREADS (16 per GPU)
    threads = int(os.environ.get("OMP_NUM_THREADS") or 0) or len(os.sched_getaffinity(0))
    threads = max(1, min(threads, len(os.sched_getaffinity(0))))
    torch.set_num_threads(threads)
    torch.manual_seed(1000)
    m = heads.ClsSSG()
    cases.randomize_bn(m, 2000)
    sd = {k: v.detach().float() for k, v in m.state_dict().items()}
    Bs, N = 32, 1024  # the metric's configuration (SSG B=32 N=1024)
    x = cases.cloud("uniform3", Bs, N, 7).permute(0, 2, 1).contiguous()
    with torch.no_grad():
        torch_ref.cls_ssg_forward(sd, x)  # warm-up
        n, t0 = 0, time.perf_counter()
        while True:
            torch_ref.cls_ssg_forward(sd, x)
            n += 1
            el = time.perf_counter() - t0
            if el >= seconds or n >= 50:
                break
    cpu = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": round(Bs * n / el, 3), "unit": "point-clouds/s", "cores": threads,
            "kind": "port",
            "sample": "oracle/torch_ref.py cls_ssg forward (reference formulation, torch %s CPU), "
                      "B=%d N=%d x %d forwards in %.1f s on %s" % (torch.__version__, Bs, N, n, el, cpu)}


def load_traffic(cfg, op="pn2_sa_mlp_max_f32"):
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as fh:
            d = json.load(fh)
        return d.get(cfg, {}).get(op)
    except (OSError, ValueError):
        return None


def load_mfma_busy(cfg):
    """MFMA-pipe busy fraction of the MLP op's kernels from the SQ counters
    (profiles/sq_mfma.json, tools/sq_mfma.sh: SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x
    1024 SIMDs), each kernel alone on the chip): per kernel, and time-weighted over them --
    the executed-products fraction of the MFMA peak beside roofline.frac's algorithmic one."""
    p = os.path.join(ROOT, "profiles", "sq_mfma.json")
    try:
        with open(p) as fh:
            d = json.load(fh).get(cfg, {})
    except (OSError, ValueError):
        return None
    mlp = {k: v for k, v in d.items()
           if any(n in k for n in ("sa_chain_kernel", "dense_split_kernel", "dense_lds_kernel", "dense_pair_kernel"))}
    if not mlp:
        return None
    t = sum(v["gui_us"] * v["calls"] for v in mlp.values())
    agg = sum(v["mfma_busy"] * v["gui_us"] * v["calls"] for v in mlp.values()) / t
    short = {k.split("(")[0].replace("void pn2::", ""): v["mfma_busy"] for k, v in mlp.items()}
    return {"time_weighted": round(agg, 4), "per_kernel": short,
            "source": "profiles/sq_mfma.json (SQ_VALU_MFMA_BUSY_CYCLES, eager launch)"}


def count_gpus(topology="/sys/class/kfd/kfd/topology/nodes"):
    """GPUs this process may use, counted without initialising HIP: the KFD topology's GPU
    nodes (simd_count > 0), capped by HIP_/ROCR_/CUDA_VISIBLE_DEVICES.  The launcher's parent
    forks its ranks afterwards, so it must not have touched the GPU runtime (torch's
    device_count() falls back to initialising HIP when amdsmi does not answer)."""
    n = 0
    try:
        for node in os.listdir(topology):
            try:
                with open(os.path.join(topology, node, "properties")) as fh:
                    props = dict(line.split(None, 1) for line in fh if line.strip())
            except (OSError, ValueError):
                continue
            if int(props.get("simd_count", "0")) > 0:
                n += 1
    except OSError:
        return 0
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([t for t in v.split(",") if t.strip()]))
    return n


def rank_envs(n, port, base=None):
    """The environment of each of n single-GPU ranks on this node (what torchrun sets)."""
    envs = []
    for r in range(n):
        e = dict(os.environ if base is None else base)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n),
                  "LOCAL_WORLD_SIZE": str(n), "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                  "MASTER_PORT": str(port), "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
        envs.append(e)
    return envs


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, cmd=None, timeout=None):
    """`bench.py --gpus N` without a launcher: start N child processes, one per GPU, each with
    the torchrun environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*), then wait.  The parent
    never touches the GPU (it only counts devices); rank 0 prints the JSON line on the shared
    stdout.  If a rank fails the others are stopped and its exit code is returned."""
    import subprocess
    cmd = cmd or [sys.executable, os.path.abspath(__file__)]
    procs = [subprocess.Popen(cmd + list(argv), env=e) for e in rank_envs(n, free_port())]
    rc, t0 = 0, time.time()
    try:
        live = list(procs)
        while live:
            for p in list(live):
                r = p.poll()
                if r is None:
                    continue
                live.remove(p)
                if r != 0 and rc == 0:
                    rc = r if r > 0 else 128 - r
                    for q in live:
                        q.terminate()
            if timeout is not None and time.time() - t0 > timeout and live:
                for q in live:
                    q.kill()
                rc = rc or 124
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


def main():
    a = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        if not a.plumbing_check:
            ndev = count_gpus()  # no HIP call in the parent: it forks the ranks next
            if ndev < a.gpus:
                sys.exit("bench.py: --gpus %d but only %d device(s) visible" % (a.gpus, ndev))
        sys.exit(launch_ranks(a.gpus, sys.argv[1:]))
    if env_world is not None and int(env_world) != a.gpus:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE=%s (the launcher started %s ranks)"
                 % (a.gpus, env_world, env_world))
    if a.plumbing_check:
        return plumbing_check(a)
    if a.hw_queues > 0:
        # HW queues per process (read by the HIP runtime at its first call, below).  The
        # pipeline keeps 4 streams busy (caller, geometry, compute, head tail); RCCL adds its own
        # streams, and with HIP's default of 4 queues two of the pipeline's streams then share
        # one: -10 % at world size 1 with the all_gather forced through RCCL (115 vs 129-131k),
        # nothing with 8 queues (131k); no change without RCCL
        os.environ["GPU_MAX_HW_QUEUES"] = str(a.hw_queues)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 or a.force_rccl:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if world == 1:  # --force-rccl: a 1-rank RCCL group of its own
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    import pn2  # noqa: F401
    from pn2 import ops, shard, tuning
    if a.force_rccl:
        # every step's all_gather of the head outputs runs through RCCL at world size 1 (the
        # collective's queue and launch cost on one GPU)
        tuning.override(force_gather=1).__enter__()
    if os.environ.get("PN2_BENCH_AFFINITY"):  # diagnostics: the host threads' CPU affinity
        print("affinity before first collective:", len(os.sched_getaffinity(0)), file=sys.stderr)

    head, B, N, kind, desc = CONFIGS[a.config]
    prec = a.precision or DEFAULT_PRECISION.get(a.config, "fp32")
    ctx = pn2.mlp_precision(prec)
    ctx.__enter__()  # for the whole run (the pipeline captures its graphs under it)
    gB = B if a.config in STRONG else B * world
    lo, hi = shard.shard_range(gB, rank, world)
    names, eager_models = build_models(a.config, dev)
    from pn2.graphs import GraphedForward
    from pn2.pipeline import PointNetSetAbstraction, PointNetSetAbstractionMsg
    has_sa = any(isinstance(mod, (PointNetSetAbstraction, PointNetSetAbstractionMsg))
                 for m in eager_models for mod in m.modules())
    if not has_sa and not a.no_pipeline:
        a.graph = True  # v1: no FPS chain to overlap; whole-forward HIP-graph replay instead
    models = [GraphedForward(m) for m in eager_models] if a.graph else eager_models
    x, mean = make_inputs(a.config, hi - lo, lo, dev, rank, gB)
    torch.manual_seed(1234)  # identical CPU RNG stream on every rank (FPS start draws)

    # single-head configs run software-pipelined (pn2.pipeline: the FPS chain of step i+1 on
    # its own CUs while step i's MLPs run); same kernels, results and RNG draws as eager steps
    pipelined = not a.graph and not a.no_pipeline
    pf = None
    if pipelined:
        from pn2.pipeline import GraphedPipeline, MultiHead, PipelinedForward
        # several heads (config pose): one module, heads in step()'s order, so the FPS draws
        # come in the same order and every head's geometry overlaps every head's MLPs
        pmodel = eager_models[0] if len(eager_models) == 1 else MultiHead(
            eager_models, [i for i, n in enumerate(names) if n.startswith("translation")])
        def graphed(gb, fuse, nslots=None):
            one = gb == 1 or not fuse  # every launch one batch (the headline)
            return GraphedPipeline(pmodel, geometry_cus=a.geometry_cus,
                                   tail=not a.no_tail,
                                   nslots=nslots if nslots is not None else max(4 * gb, DEFAULT_SLOTS),
                                   geometry_streams=(a.geometry_streams if a.geometry_streams is not None
                                                     else 4 if one else
                                                     DEFAULT_GEOMETRY_STREAMS.get(a.config, 1)),
                                   geometry_batches=gb, fuse=fuse,
                                   compute_streams=a.compute_streams,
                                   geometry_bq=(bool(a.geometry_bq) if a.geometry_bq is not None
                                                else False if one else None),
                                   tail_streams=2 if one else None)

        if not a.eager_pipeline:
            pf = graphed(a.geometry_batches, a.fuse, a.slots)
        else:
            pf = PipelinedForward(pmodel, geometry_cus=a.geometry_cus,
                                  tail="auto" if a.tail else False)

    takes_mean = any(n.startswith("translation") for n in names)

    def gather(i, o):  # step()'s all_gather of every head's first output
        if len(names) > 1:
            return [shard.all_gather_rows(h[0] if isinstance(h, tuple) else h, sizes="shard")
                    for h in o]
        return shard.all_gather_rows(o[0] if isinstance(o, tuple) else o, sizes="shard")

    def first_outputs(o):  # every head's first output (the logits / predictions)
        if len(names) > 1:
            return [h[0] if isinstance(h, tuple) else h for h in o]
        return o[0] if isinstance(o, tuple) else o

    def run_pipelined(k, pf_=None):
        pf_ = pf_ or pf
        with shard.batch_shard(gB, lo):
            if a.gather_every > 1:  # one collective per gather_every batches
                bg = shard.BatchedGather(a.gather_every, total=k)
                post = lambda i, o: bg(i, first_outputs(o))  # noqa: E731
            else:
                post = gather
            pf_.run([x] * k, [(mean,)] * k if takes_mean else None, post=post)

    for _ in range(max(a.warmup, 2) if a.graph else a.warmup):  # graph: 1st call captures
        step(names, models, x, mean, gB, lo)
    if pipelined:
        run_pipelined(max(a.warmup, 2))
    torch.cuda.synchronize()
    if os.environ.get("PN2_BENCH_AFFINITY"):
        import threading
        print("affinity after warmup:", len(os.sched_getaffinity(0)), "threads:",
              threading.active_count(), "os threads:", len(os.listdir("/proc/self/task")), file=sys.stderr)

    def timed(k, timer, models=models, pipe=False):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if pipe:
            kt = None
            run_pipelined(k, pipe if pipe is not True else None)
        elif timer:
            with ops.kernel_timer() as kt:
                for _ in range(k):
                    step(names, models, x, mean, gB, lo)
                torch.cuda.synchronize()
        else:
            kt = None
            for _ in range(k):
                step(names, models, x, mean, gB, lo)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if world > 1:
            dist.barrier()
        return el, kt

    def max_over_ranks(el):
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    el, _ = timed(a.steps, False, pipe=pipelined)
    el = max_over_ranks(el)
    ms = el / a.steps * 1e3
    value = gB * a.steps / el
    eager_value = value
    # The same K batches again once the device has been busy for a while (untimed pipelined
    # batches for ~80 ms first): after an idle gap the SOC clock sits in deep sleep (38-47 MHz)
    # and needs ~30 ms of load to reach 1200 MHz, and a pipelined run at a low SOC clock is up
    # to 25 % slower (tools/debug/clock_trace.py).  `value` above is the
    # contract's number (W warm-up steps, then K timed); this one is reported beside it.
    settled = None
    if pipelined and not a.no_settled:
        run_pipelined(max(a.steps, int(80.0 / max(ms, 1e-3)) + 1))
        el_s, _ = timed(a.steps, False, pipe=True)
        el_s = max_over_ranks(el_s)
        settled = {"value": round(gB * a.steps / el_s, 2), "ms_per_step": round(el_s / a.steps * 1e3, 4),
                   "settle": "~80 ms of untimed pipelined batches before the same K timed steps"}
    # The same K batches through a pipeline that fuses `fused_batches` consecutive batches into
    # every launch (FPS over their clouds side by side, one forward over all their rows): a
    # serving mode with launch batch fused_batches x B, bit-equal per batch to the eager forward
    # (tests/test_gpu_configs.py), reported beside the headline, never as it.
    fused = None
    if pipelined and not a.eager_pipeline and a.fused_batches > 1 and (
            a.fuse is False or a.geometry_batches != a.fused_batches):
        pf4 = graphed(a.fused_batches, True)
        run_pipelined(max(a.warmup, 2), pf4)
        run_pipelined(max(a.steps, int(80.0 / max(ms, 1e-3)) + 1), pf4)
        el_f, _ = timed(a.steps, False, pipe=pf4)
        el_f = max_over_ranks(el_f)
        fused = {"value": round(gB * a.steps / el_f, 2), "ms_per_step": round(el_f / a.steps * 1e3, 4),
                 "launch_batch": a.fused_batches * (hi - lo), "geometry_batches": a.fused_batches,
                 "launch": "graphed pipeline; %d consecutive batches per launch (FPS, ball queries, "
                           "MLPs, head), after ~80 ms of untimed batches" % a.fused_batches}
        del pf4
    if a.graph or pipelined:
        # the eager pass's own warm-up: after the pipelined runs (whose graphs keep private
        # memory pools) the first eager forwards allocate afresh
        for _ in range(3):
            step(names, eager_models, x, mean, gB, lo)
        el_e, _ = timed(a.steps, False, eager_models)
        eager_value = gB * a.steps / max_over_ranks(el_e)
    # The unchanged reference head through the drop-in: its forward restated call for call
    # (pn2.heads.ReferenceForward -- SA modules one after the other, no FPS side job, the torch
    # FC tail), eager, the same K steps
    ref_value = None
    if not a.no_reference_head:
        from pn2 import heads as _heads
        if all(n in _heads.HEADS for n in names):
            ref_models = [_heads.ReferenceForward(m) for m in eager_models]
            for _ in range(3):
                step(names, ref_models, x, mean, gB, lo)
            el_r, _ = timed(a.steps, False, ref_models)
            ref_value = round(gB * a.steps / max_over_ranks(el_r), 2)
    kt = None
    if not a.no_kernel_timer:
        _, kt = timed(a.steps, True, eager_models)

    kern = kt.summary() if kt is not None else {}
    mlp_name = "pn2_sa_mlp_max_bf16" if prec == "bf16" else "pn2_sa_mlp_max_f32"
    mlp = kern.get(mlp_name)
    roof = None
    if mlp and mlp["ms"] > 0:
        achieved = mlp["flops"] / (mlp["ms"] * 1e-3) / 1e12
        # the ceiling of the mix the calls ran: sum(flops) / sum(flops_i / peak_i) -- the rate
        # at which every call at its own arithmetic's MFMA peak would do the same work
        fbp = {p: f for p, f in mlp["flops_by_planes"].items() if PEAK_BY_PLANES.get(p)}
        if fbp:
            peak = sum(fbp.values()) / sum(f / PEAK_BY_PLANES[p] for p, f in fbp.items())
        else:
            peak = PEAK_BF16_MFMA if prec == "bf16" else PEAK_SPLIT
        mix = {{3: "split bf16 x6", 2: "split fp16 x3", 1: "bf16 x1", 0: "fp32"}[p]:
               round(f / mlp["flops"], 4) for p, f in sorted(mlp["flops_by_planes"].items())}
        roof = {"bound": "mfma", "achieved": round(achieved, 3), "peak": round(peak, 1),
                "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                "peak_basis": "flops-weighted MFMA ceiling of the arithmetic each call ran: split "
                              "fp16 %.1f, split bf16 %.1f, bf16 %.1f TFLOP/s fp32-equivalent" % (
                                  PEAK_BF16_MFMA / 3, PEAK_BF16_MFMA / 6, PEAK_BF16_MFMA),
                "flops_mix": mix,
                "frac_vs_split_bf16_ceiling": round(achieved / PEAK_SPLIT, 4),
                "traffic": load_traffic(a.config, mlp_name),
                "compulsory_bytes_per_launch": mlp["bytes"] / mlp["launches"],
                "kernel": "%s (sa_chain_kernel / dense_split_kernel, %s)" % (
                    mlp_name, "bf16, 1 MFMA per product" if prec == "bf16" else
                    "fp32-accurate split fp16 (chains, dense hidden layers) / split bf16 (first dense "
                    "layer, streamed chain inputs)"),
                "fp32_mfma_peak": PEAK_F32_MFMA,
                "frac_of_fp32_mfma_peak": round(achieved / PEAK_F32_MFMA, 4),
                "flops_per_launch": mlp["flops"] / mlp["launches"],
                "flops_basis": "algorithmic: 2*M*sum(cin*cout) per call over all B*S*K grouped "
                               "rows (the reference's conv work); the kernels execute fewer "
                               "products (layer 0 once per source point on wide first layers, "
                               "only each group's distinct neighbour rows), so achieved and "
                               "frac are effective rates",
                "avg_launch_ms": mlp["ms"] / mlp["launches"]}
        roof["mfma_busy"] = load_mfma_busy(a.config)
        if roof["traffic"]:
            roof["traffic_vs_compulsory"] = round(roof["traffic"] / roof["compulsory_bytes_per_launch"], 2)
    kernels = {k: {"ms_per_step": round(v["ms"] / a.steps, 4), "launches_per_step": v["launches"] / a.steps}
               for k, v in kern.items()}
    # the north star's named kernel, query_ball_point: VALU-bound under compulsory-byte
    # accounting; its HBM fraction is reported beside the VALU one
    bq = kern.get("pn2_ball_query_f32")
    roof_bq = None
    if bq and bq["ms"] > 0:
        t = bq["ms"] * 1e-3
        roof_bq = {"bound": "valu", "achieved": round(bq["flops"] / t / 1e12, 3), "peak": PEAK_F32_VALU,
                   "unit": "TFLOP/s", "frac": round(bq["flops"] / t / 1e12 / PEAK_F32_VALU, 4),
                   "hbm_achieved": round(bq["bytes"] / t / 1e9, 1), "hbm_peak": PEAK_HBM,
                   "hbm_unit": "GB/s", "hbm_frac": round(bq["bytes"] / t / 1e9 / PEAK_HBM, 4),
                   "traffic": load_traffic(a.config, "pn2_ball_query_f32"),
                   "kernel": "pn2_ball_query_f32 (ball_query_kernel)",
                   "flops_basis": "algorithmic: every centroid-point pair x (2C+3) (SURVEY 8(d)); the "
                                  "kernel stops a cloud's scan once all its centroids have K hits",
                   "bytes_basis": "compulsory: packed points and centroids in, the SA path's "
                                  "int32 [B,S,K] lists and [B,S] counts out",
                   "avg_launch_ms": bq["ms"] / bq["launches"]}

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline and a.config == "ssg":
        cpu = cpu_baseline(a.cpu_seconds)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "point-clouds/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "strong" if a.config in STRONG else "weak", "vs_baseline": None,
            "dtype": ("bf16 (MLP operands bf16, fp32 accumulate / BN / max; FPS/ball query f32)"
                      if prec == "bf16" else
                      "f32 (MLP products fp32-accurate: split fp16 x3 in the chains and the dense "
                      "hidden layers, split bf16 x6 in the first dense layers, fp32 accumulate; "
                      "FPS/ball query f32)"),
            "data": "synthetic: seeded uniform clouds normalised to the unit sphere%s; seeded "
                    "random-init weights and BN statistics (eval mode)" % (
                        " + 7-way one-hot" if kind == "onehot10" else ""),
            "config": {"workload": desc, "global_batch": gB, "points": N, "heads": names,
                       "launch_batch": (hi - lo) * (a.geometry_batches if pipelined and a.fuse else 1),
                       "parallelism": "dp%d" % world + (" (all_gather forced through RCCL)"
                                                         if a.force_rccl else "")},
            "roofline": roof, "roofline_ball_query": roof_bq, "cpu_baseline": cpu, "kernels": kernels,
            "launch": ("hip_graph" if a.graph else
                       "%s pipeline (fps%s stream%s)" % (
                           "eager" if a.eager_pipeline else "graphed",
                           " + head" if (not a.eager_pipeline and not a.no_tail) or (
                               a.tail and not names[0].startswith("translation")) else "",
                           " on %d dedicated CUs" % a.geometry_cus if a.geometry_cus > 0
                           else "s sharing all CUs") + (
                           "; geometry of %d batches per replay" % a.geometry_batches +
                           ("; one forward per geometry group" if getattr(pf, "_slots", None) and
                            pf._slots[0].halves[0].fused else "; one forward per batch") +
                           ("; %d compute + %d geometry + %d tail streams%s%s" % (
                               pf.compute_streams, pf.geometry_streams, pf.tail_streams,
                               "" if pf.head_on_tail else ", heads on the compute streams",
                               "; ball queries in each batch's forward" if pf.geometry_bq is False else ""))
                           if not a.eager_pipeline else "")
                       if pipelined else "eager"),
            "eager_value": round(eager_value, 2),
            "eager_value_reference_head": ref_value,
            "value_fused": fused,
            "value_settled": settled,
            # hardware queues of this process (bench.py sets 8 unless --hw-queues 0; HIP's own
            # default is 4: DESIGN.md §6)
            "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "HIP default (4)"),
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
