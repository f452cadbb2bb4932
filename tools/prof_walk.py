"""Walker timing breakdown from the SALN_WALK_PROF build (libsaln_prof.so):
shader cycles per walk, in window waits and in synchronous refills."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sequencealigning_amd import _lib  # noqa: E402

_lib.LIB_PATH = _lib.LIB_PATH.replace("libsaln.so", "libsaln_prof.so")


def main():
    import torch
    import sequencealigning_amd as saln
    from sequencealigning_amd import synth
    n, L = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000, 150
    qs, qo, ds, do = synth.iid_pairs(n, L, L, seed=0x5EED0002)
    plan = saln.NwPlan(qo, do, pairs=np.stack([np.arange(n)] * 2, 1))
    dq, dd = torch.from_numpy(qs).cuda(), torch.from_numpy(ds).cuda()
    res = torch.zeros(n * 4, dtype=torch.int32, device="cuda")
    for _ in range(3):
        plan.execute(dq, dd, res, None)
    torch.cuda.synchronize()
    r = res.cpu().numpy().reshape(n, 4)
    tot = r[:, 0].astype(np.float64) * 16
    wait = r[:, 1].astype(np.float64) * 16
    sync = (r[:, 2].astype(np.uint32)).astype(np.float64) * 16
    flags = (r[:, 3] >> 8) & 0xFF
    iters = ((r[:, 3] >> 24) & 0xFF) * 4
    print(f"pairs {n}: cycles/walk mean {tot.mean():.0f} max {tot.max():.0f}")
    print(f"  window wait {wait.mean():.0f} ({wait.mean() / tot.mean():.1%}), "
          f"phase ends {sync.mean():.0f} ({sync.mean() / tot.mean():.1%}) n={flags.mean():.2f}")
    print(f"  lane iterations ~{iters.mean():.0f}; cycles/iteration {tot.mean() / max(1, iters.mean()):.0f}")


if __name__ == "__main__":
    main()
