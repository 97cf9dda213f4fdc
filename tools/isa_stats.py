"""Static instruction mix of device functions in a hipcc -S listing (gfx950).
usage: python tools/isa_stats.py engine.s REGEX   (e.g. k_whatif_rec1)"""
import re
import sys
from collections import Counter

src = open(sys.argv[1]).read()
pat = re.compile(sys.argv[2])
for m in re.finditer(r"^(_Z\w+):\s*;.*?$(.*?)^\.Lfunc_end\d+:", src, re.S | re.M):
    name, body = m.group(1), m.group(2)
    if not pat.search(name):
        continue
    c = Counter()
    for line in body.split("\n"):
        t = line.strip()
        if not t or t[0] in ".;" or t.endswith(":"):
            continue
        op = t.split()[0]
        if op.startswith("s_waitcnt") or op in ("s_nop",):
            c["wait/nop"] += 1
        elif op.startswith(("s_load", "s_buffer_load")):
            c["smem"] += 1
        elif op.startswith("s_"):
            c["salu/branch"] += 1
        elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
            c["vmem"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
            c["lane"] += 1
        elif op.startswith("v_"):
            c["valu"] += 1
        else:
            c[op] += 1
    tail = src[m.end():m.end() + 4000]
    meta = {k: re.search(r"; %s: (\S+)" % k, tail) for k in ("NumVgprs", "NumSgprs", "ScratchSize", "Occupancy")}
    print(name[:70], dict(c), {k: v.group(1) for k, v in meta.items() if v})
