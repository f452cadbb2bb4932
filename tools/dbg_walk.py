import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sequencealigning_amd import _lib
_lib.LIB_PATH = _lib.LIB_PATH.replace("libsaln.so", "libsaln_dbg.so")
import sequencealigning_amd as saln
vecs = json.load(open("tests/golden/nw_random.json"))["pairs"]
res, cig = saln.nw_align_batch([v["query"].encode() for v in vecs], [v["db"].encode() for v in vecs],
                               pairs=[(k, k) for k in range(len(vecs))], with_cigar=False)
n = 0
for k in range(len(vecs)):
    if res["flags"][k] & 4:
        n += 1
        info = int(res["cigar_len"][k])
        if n < 12:
            print(k, "mismatches", int(res["reserved"][k]), "S", info & 7, "par", (info >> 3) & 1,
                  "valid", (info >> 4) & 1, "ti", (info >> 8) & 0xFFF, "tj", (info >> 20) & 0xFFF,
                  "lq", len(vecs[k]["query"]), "ld", len(vecs[k]["db"]))
print("pairs with mismatches:", n)
