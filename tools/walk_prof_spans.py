import sys, os, time, ctypes as C
sys.path.insert(0, os.getcwd())
import numpy as np, torch
import sequencealigning_amd as saln
from sequencealigning_amd import synth, _lib
from sequencealigning_amd import span as S
q = synth.random_bases(0x5EED0003, 100_000).tobytes()
d = synth.mutate(q, 0.05, seed=100_000)
ch = S.SpanChain(q, d, 8, band_rows=1024)
for it in range(3):
    ch.fill(True); torch.cuda.synchronize()
    t0 = time.perf_counter(); ch.check(); t1 = time.perf_counter()
    sc, st = ch.spans[-1].score(); t2 = time.perf_counter()
    L = _lib.lib()
    hs = (C.c_void_p * 8)(*[s._h.value for s in ch.spans]); cap = len(q) + len(d) + 16
    buf = (C.c_uint32 * cap)(); ex, n = _lib.SpanCursor(), C.c_uint64()
    rc = L.saln_nw_spans_walk(hs, 8, C.c_void_p(ch.q.data_ptr()), C.c_void_p(ch.d.data_ptr()), C.byref(ex), buf, cap, C.byref(n), _lib.torch_stream(0))
    t3 = time.perf_counter()
    ops = np.ctypeslib.as_array(buf)[:n.value].copy()
    cig = S.merge_walk_ops([ops]); t4 = time.perf_counter()
    print(f"rc={rc} nops={n.value} runs={len(cig)} check={1e3*(t1-t0):.3f} score={1e3*(t2-t1):.3f} spanswalk={1e3*(t3-t2):.3f} merge={1e3*(t4-t3):.3f} ms", flush=True)
ch.close()
