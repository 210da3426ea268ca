"""Instruction histogram of one kernel in a hipcc -S listing, per basic block.

  hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S edv_verify.hip -o /tmp/edv.s
  python tools/isa_hist.py /tmp/edv.s edv_main_kernel [top]

Prints the kernel's total static instruction count, the largest basic blocks
(the main loop body is the one that matters for the issue-bound kernels) and
the opcode histogram of the largest block.
"""
import collections
import re
import sys


def kernel_body(text, name):
    m = re.search(r"^(\S*%s\S*):" % re.escape(name), text, re.M)
    if not m:
        raise SystemExit("kernel %s not found" % name)
    body = text[m.end():]
    return body[:body.index(".Lfunc_end")]


def blocks(body):
    cur, out = "entry", collections.OrderedDict()
    out[cur] = []
    for line in body.splitlines():
        s = line.strip()
        if not s or s.startswith((";", ".")) and not s.startswith(".LBB"):
            continue
        if s.endswith(":") or re.match(r"^\.LBB\S*:", s):
            cur = s.split(":")[0]
            out[cur] = []
            continue
        op = s.split()[0]
        if op.startswith((".", ";")):
            continue
        out[cur].append(op)
    return out


def main():
    text = open(sys.argv[1]).read()
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    bb = blocks(kernel_body(text, sys.argv[2]))
    print("total static instructions:", sum(len(v) for v in bb.values()))
    big = sorted(bb.items(), key=lambda kv: -len(kv[1]))[:6]
    for k, v in big:
        print("  block %-12s %6d" % (k, len(v)))
    k, v = big[0]
    c = collections.Counter(v)
    print("histogram of %s:" % k)
    for op, n in c.most_common(top):
        print("  %6d %s" % (n, op))


if __name__ == "__main__":
    main()
