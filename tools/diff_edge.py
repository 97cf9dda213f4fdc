"""Debug aid: first pod where the engine and the oracle disagree on an edge
variant, with the per-node score / finalscore / filter differences.
usage: python tools/diff_edge.py VARIANT [cycle]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-scheduler-simulator-p9_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch  # noqa: F401
    from _oracle import Oracle
    from ksg import Scheduler, edge
    v = sys.argv[1]
    cyc = len(sys.argv) > 2
    doc = edge.generate_edge(v)
    o = Oracle(doc)
    o.schedule(record=3)
    s = Scheduler(doc["profile"])
    if cyc:
        d = dict(doc)
        d["queue"] = []
        s.load_cluster(d)
    else:
        s.load_cluster(doc)
        s.keep_outputs(0, s.queue_len)
        s.schedule()
    P = "kube-scheduler-simulator.sigs.k8s.io/"
    for i, pod in enumerate(doc["queue"]):
        if cyc:
            q, r = s.cycle(pod, commit=True)
        else:
            q, r = i, s.results(i, 1)[0]
        if (r.selected, r.feasible, r.status) == o.result(i) and s.annotations(q) == o.annotations(i):
            continue
        print("pod", i, "engine", (r.selected, r.feasible, r.status), "oracle", o.result(i))
        print("spec", json.dumps(pod["spec"])[:1500])
        a, b = s.annotations(q), o.annotations(i)
        for k in b:
            if a.get(k) != b[k]:
                ka, kb = json.loads(a[k]) if a.get(k, "").startswith("{") else a.get(k), \
                    json.loads(b[k]) if b[k].startswith("{") else b[k]
                if isinstance(ka, dict) and isinstance(kb, dict):
                    n = 0
                    for node in sorted(set(ka) | set(kb)):
                        if ka.get(node) != kb.get(node):
                            print(" ", k[len(P):], node, "engine", ka.get(node), "oracle", kb.get(node))
                            nd = next((x for x in doc["nodes"] if x["metadata"]["name"] == node), None)
                            if nd is not None and n == 0:
                                print("    node", json.dumps(nd)[:600])
                            n += 1
                            if n >= 4:
                                break
                else:
                    print(" ", k[len(P):], "engine", str(ka)[:300], "oracle", str(kb)[:300])
        break


if __name__ == "__main__":
    main()
