"""Per-kernel ISA stats from `make asm` output (scratch use, waitcnts, VGPRs)."""
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "sequencealigning_amd/build/nw_kernels.s"
pat = sys.argv[2] if len(sys.argv) > 2 else ""
s = open(path).read()
for m in re.finditer(r'^(_Z\S*):[^\n]*\n(.*?)\.Lfunc_end', s, re.S | re.M):
    name, body = m.group(1), m.group(2)
    if pat not in name:
        continue
    vg = re.search(r'\.set ' + re.escape(name) + r'\.num_vgpr, (\d+)', s)
    sc = re.search(r'\.set ' + re.escape(name) + r'\.private_seg_size, (\d+)', s)
    print(f"{name[:70]:70s} lines={body.count(chr(10)):5d} scratch_ops={body.count('scratch_'):3d} "
          f"vmcnt={len(re.findall(r'vmcnt', body)):3d} vmcnt0={len(re.findall(r'vmcnt[(]0[)]', body)):3d} "
          f"vgpr={vg.group(1) if vg else '?'} priv={sc.group(1) if sc else '?'}")
