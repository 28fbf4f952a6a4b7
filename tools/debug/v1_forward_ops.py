import os, sys, torch
ROOT="/root/repo"
sys.path[:0]=[ROOT+"/pointnet-like-pose-estimation_amd", ROOT+"/tests/golden"]
import cases
from pn2.heads_v1 import PointNetCls
m=PointNetCls().cuda().eval()
x=cases.cloud("uniform3",8,1024,5).permute(0,2,1).contiguous().cuda()
with torch.no_grad():
    for _ in range(3): m(x)
    torch.cuda.synchronize()
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        m(x); torch.cuda.synchronize()
print(prof.key_averages(group_by_stack_n=0).table(sort_by="cpu_time_total", row_limit=45))
