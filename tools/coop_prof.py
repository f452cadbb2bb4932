import os, sys, numpy as np
sys.path.insert(0, os.getcwd())
import torch
import sequencealigning_amd as saln
from sequencealigning_amd import synth
L = int(sys.argv[1])
q = synth.random_bases(0x5EED0003, L).tobytes()
d = synth.mutate(q, 0.05, seed=L)
qs, qo = saln.pack_csr([q]); ds, do = saln.pack_csr([d])
plan = saln.NwPlan(qo, do, pairs=np.array([[0, 0]]))
dq, dd = torch.from_numpy(qs).cuda(), torch.from_numpy(ds).cuda()
res = torch.zeros(4, dtype=torch.int32, device="cuda")
cig = torch.zeros(max(1, plan.cigar_words), dtype=torch.int32, device="cuda")
for _ in range(2):
    plan.execute(dq, dd, res, cig)
torch.cuda.synchronize()
r = res.cpu().numpy()
print("L", L, "loads", r[0], "clk>>10 total", r[1], "iters", r[2], "load%", (r[3] >> 24) & 0xFF, "emit%", r[3] & 0xFF)
