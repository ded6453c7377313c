"""Read a HIP graph DOT dump (tools/graph_dot.py) and report, for a kernel
node matching PATTERN, which kernels precede it in the graph (its ancestors),
and its direct predecessors -- to check that the captured step's branches
carry only the dependencies the code asked for.
    python tools/graph_edges.py gpurun_out/graph/step_0.dot wr_fwd_pipe"""
import re
import sys
from collections import defaultdict


def load(path):
    text = open(path).read()
    labels, preds = {}, defaultdict(set)
    for m in re.finditer(r'"?([\w]+)"?\s*\[([^\]]*)\]', text):
        lab = re.search(r'label\s*=\s*"((?:[^"\\]|\\.)*)"', m.group(2))
        if lab:
            labels[m.group(1)] = lab.group(1)
    for m in re.finditer(r'"?([\w]+)"?\s*->\s*"?([\w]+)"?', text):
        preds[m.group(2)].add(m.group(1))
    return labels, preds


def short(label):
    k = re.search(r"(\w+_kernel\w*|\w+Kernel\w*|\w+elementwise\w*|memset\w*|memcpy\w*|event\w*)",
                  label)
    return k.group(1) if k else label[:60]


def main(path, pattern):
    labels, preds = load(path)
    hits = [n for n, l in labels.items() if pattern in l]
    print(f"{len(labels)} nodes, {sum(len(v) for v in preds.values())} edges; "
          f"{len(hits)} node(s) match {pattern!r}")
    for n in hits:
        seen, stack = set(), [n]
        while stack:
            for p in preds[stack.pop()]:
                if p not in seen:
                    seen.add(p)
                    stack.append(p)
        print(f"\n{n}: direct preds: {sorted(short(labels.get(p, p)) for p in preds[n])}")
        names = sorted({short(labels.get(p, p)) for p in seen})
        print(f"  {len(seen)} ancestors; kernels: {names}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
