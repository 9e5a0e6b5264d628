"""Synthetic rule-set generators for the bench/parity configs (fixture specs).

These are the exact recipes of SURVEY.md Appendix A (configs B, C, E).  They
use CPython's ``random.Random(seed)`` whose sequence is stable across 3.x, so
the generated rule text -- and therefore the Aho-Corasick tables libyara builds
from it -- is reproducible here and on the GPU box.

    python tests/golden/gen_rules.py B > b.yar      # 1k 4-byte hex literals
    python tests/golden/gen_rules.py C > c.yar      # 10k mixed hex/ascii/wildcard
    python tests/golden/gen_rules.py E > e.yar      # 2k nocase + nibble wildcards
"""
import random
import sys

ALNUM = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789_"


def gen_bc(n: int, mode: str, seed: int) -> str:
    r = random.Random(seed)
    out = []
    per = 100
    for k in range(0, n, per):
        out.append("rule r%d {\n strings:" % (k // per))
        for j in range(k, min(n, k + per)):
            if mode == "lit4":
                b = bytes(r.getrandbits(8) for _ in range(4))
                out.append("  $s%d = { %s }" % (j, " ".join("%02X" % x for x in b)))
            else:
                t = j % 3
                if t == 0:
                    L = r.randint(4, 16)
                    b = bytes(r.getrandbits(8) for _ in range(L))
                    out.append("  $s%d = { %s }" % (j, " ".join("%02X" % x for x in b)))
                elif t == 1:
                    L = r.randint(4, 12)
                    s = "".join(r.choice(ALNUM) for _ in range(L))
                    out.append('  $s%d = "%s"' % (j, s))
                else:
                    L = r.randint(2, 6)
                    b = ["%02X" % r.getrandbits(8) for _ in range(L)]
                    b.insert(r.randint(1, L - 1), "??")
                    b2 = ["%02X" % r.getrandbits(8) for _ in range(3)]
                    out.append("  $s%d = { %s [1-8] %s }" % (j, " ".join(b), " ".join(b2)))
        out.append(" condition: any of them\n}")
    return "\n".join(out) + "\n"


def gen_e(n: int = 2000, seed: int = 5) -> str:
    r = random.Random(seed)
    out = []
    for k in range(0, n, 100):
        out.append("rule n%d {\n strings:" % (k // 100))
        for j in range(k, k + 100):
            if j % 2 == 0:
                L = r.randint(6, 12)
                s = "".join(r.choice("abcdefghijklmnopqrstuvwxyz") for _ in range(L))
                out.append('  $s%d = "%s" nocase' % (j, s))
            else:
                b = ["%02X" % r.getrandbits(8) for _ in range(r.randint(3, 5))]
                b.insert(r.randint(1, len(b) - 1), "??")
                b.insert(r.randint(1, len(b) - 1), "%X?" % r.getrandbits(4))
                tail = " ".join("%02X" % r.getrandbits(8) for _ in range(4))
                out.append("  $s%d = { %s [2-16] %s }" % (j, " ".join(b), tail))
        out.append(" condition: any of them\n}")
    return "\n".join(out) + "\n"


def gen(config: str) -> str:
    if config == "B":
        return gen_bc(1000, "lit4", 1)
    if config == "C":
        return gen_bc(10000, "mixed", 2)
    if config == "E":
        return gen_e()
    raise ValueError(config)


if __name__ == "__main__":
    sys.stdout.write(gen(sys.argv[1]))
