"""Drop-in cycle latency at the C ABI: builds tools/dropin_harness.c against the
in-tree libksg.so, writes a BASELINE config's profile, cluster (empty queue) and a
stream of its queue pods, and runs the harness (no Python in the timed calls).

usage: python tools/dropin_c.py [--cfg 2|4] [--warmup 20] [--count 200] [--out FILE]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "kube-scheduler-simulator-p9_amd")
sys.path.insert(0, PKG)


def build(exe):
    src = os.path.join(ROOT, "tools", "dropin_harness.c")
    if os.path.exists(exe) and os.path.getmtime(exe) >= os.path.getmtime(src):
        return exe
    subprocess.check_call(["gcc", "-O2", "-o", exe, src, "-I", os.path.join(ROOT, "include"), "-L", PKG, "-lksg",
                           "-ldl", f"-Wl,-rpath,{PKG}"])
    return exe


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--count", type=int, default=200)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from ksg import generator as g
    doc = json.loads(g.generate_native(a.cfg))
    pods = doc["queue"][:a.warmup + a.count]
    doc["queue"] = []
    with tempfile.TemporaryDirectory() as d:
        exe = build(os.path.join(d, "dropin_harness"))
        paths = {k: os.path.join(d, k) for k in ("profile.json", "cluster.json", "pods.jsonl")}
        json.dump(doc["profile"], open(paths["profile.json"], "w"))
        json.dump(doc, open(paths["cluster.json"], "w"))
        with open(paths["pods.jsonl"], "w") as f:
            for i, p in enumerate(pods):
                p["metadata"]["name"] = f"dropin-{i:05d}"
                f.write(json.dumps(p) + "\n")
        out = subprocess.run([exe, paths["profile.json"], paths["cluster.json"], paths["pods.jsonl"], str(a.warmup),
                              str(a.count)], capture_output=True, text=True, timeout=600)
    if out.returncode != 0:
        sys.stderr.write(out.stderr)
        sys.exit(out.returncode)
    r = json.loads(out.stdout.strip().splitlines()[-1])
    r["workload"] = f"cfg{a.cfg}"
    line = json.dumps(r)
    print(line)
    if a.out:
        with open(a.out, "a") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
