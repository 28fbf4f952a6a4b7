"""Node counts of the graphed pipeline's captured graphs (SSG): how many kernel / memcpy / memset
/ other nodes one batch costs the command processor.  The pipeline's CUDAGraphs are created
with keep_graph=True (a patch of torch.cuda.CUDAGraph for this process only) so that
hipGraphGetNodes can walk them after the first run.  python tools/debug/graph_nodes.py"""
import collections
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402,F401  (its sys.path setup)
import cases  # noqa: E402
from pn2 import heads as H  # noqa: E402
from pn2 import shard  # noqa: E402

DEV = torch.device("cuda", 0)
TYPES = {0: "kernel", 1: "memcpy", 2: "memset", 3: "host", 4: "graph", 5: "empty", 6: "wait_event",
         7: "event_record", 8: "ext_sem_signal", 9: "ext_sem_wait", 10: "mem_alloc", 11: "mem_free"}

_Orig = torch.cuda.CUDAGraph


def _keep(*a, **k):
    k["keep_graph"] = True
    return _Orig(*a, **k)


def nodes(hip, graph):
    g = ctypes.c_void_p(graph)
    n = ctypes.c_size_t(0)
    assert hip.hipGraphGetNodes(g, None, ctypes.byref(n)) == 0
    arr = (ctypes.c_void_p * n.value)()
    assert hip.hipGraphGetNodes(g, arr, ctypes.byref(n)) == 0
    c = collections.Counter()
    for i in range(n.value):
        t = ctypes.c_int(-1)
        hip.hipGraphNodeGetType(ctypes.c_void_p(arr[i]), ctypes.byref(t))
        c[TYPES.get(t.value, str(t.value))] += 1
    return n.value, dict(c)


def main():
    hip = ctypes.CDLL("libamdhip64.so")
    torch.cuda.CUDAGraph = _keep
    from pn2.pipeline import GraphedPipeline
    torch.manual_seed(8)
    model = H.ClsSSG().eval()
    cases.randomize_bn(model, 8)
    model = model.to(DEV)
    x = cases.cloud("uniform3", 32, 1024, 90).permute(0, 2, 1).contiguous().to(DEV)
    torch.manual_seed(1234)
    gp = GraphedPipeline(model)
    with shard.batch_shard(32, 0):
        gp.run([x] * 10, post=lambda i, o: shard.all_gather_rows(o[0], sizes="shard"))
    torch.cuda.synchronize()
    grp = gp._slots[0]
    tot = 0
    n, c = nodes(hip, grp.fps.raw_cuda_graph())
    print("geometry graph (%d batches): %d nodes %s" % (gp.gb, n, c))
    tot += n / gp.gb
    for h, sl in enumerate(grp.halves):
        n, c = nodes(hip, sl.sa.raw_cuda_graph())
        print("batch %d sa graph: %d nodes %s" % (h, n, c))
        tot += n / len(grp.halves)
        if sl.head is not None:
            n, c = nodes(hip, sl.head.raw_cuda_graph())
            print("batch %d head graph: %d nodes %s" % (h, n, c))
            tot += n / len(grp.halves)
    print("graph nodes per batch: %.1f (plus the host-issued copies, event records and waits)" % tot)


if __name__ == "__main__":
    main()
