"""Per-tile instruction mix of the scan kernel's main tile loop, read from the
assembly `make -C yara_amd/csrc asm` leaves (tools/isa_budget.py's sibling for
the round-6 loop shape): the common path only -- every conditional branch not
taken (the rare paths: ring full / deferred drain, no appending lane), the
unconditional ones followed -- from the loop header back to it, divided by
the tiles per iteration.

    python tools/loop_mix.py [--kernel 0] [--asm file.s] [--tiles 2]
"""
import argparse
import collections
import json
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def mix(asm, kernel, tiles):
    s = open(asm).read()
    name = "_ZN4yamd20scan_segments_kernelILi%dEEEvNS_10ScanParamsE" % kernel
    st = s.index(name + ":")
    L = s[st:s.index(".Lfunc_end", st)].splitlines()
    h = [i for i, l in enumerate(L) if "This Loop Header: Depth=2" in l][0]
    lab = {l.split(":")[0]: i for i, l in enumerate(L) if re.match(r"^\.LBB\d+_\d+:", l)}
    c = collections.Counter()
    i = h + 1
    for _ in range(4000):
        if i == h:
            break
        t = L[i].strip()
        i += 1
        if re.match(r"^\.LBB\d+_\d+:", t) and lab[t.split(":")[0]] == h:
            break
        if not t or t.startswith(";") or t.startswith("."):
            continue
        op = t.split()[0]
        if op == "s_branch":
            c["branch taken"] += 1
            i = lab[t.split()[1]]
            continue
        if op.startswith("s_cbranch"):
            c["branch not taken"] += 1
            continue
        if op.startswith("v_"):
            k = ("VALU dpp" if "dpp" in t else "VALU sdwa" if "_sdwa" in op
                 else "VALU e32 (VOP1/VOP2/VOPC)" if op.endswith("_e32") else "VALU vop3")
        elif op.startswith("s_waitcnt"):
            k = "s_waitcnt"
        elif op in ("s_nop", "s_setprio"):
            k = op
        elif op.startswith("s_"):
            k = "SALU"
        elif op.startswith("ds_"):
            k = "LDS " + op
        elif op.startswith(("buffer_", "global_")):
            k = "VMEM"
        else:
            k = op
        c[k] += 1
    return {k: round(v / tiles, 2) for k, v in sorted(c.items())}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", type=int, default=0)
    ap.add_argument("--asm", default=os.path.join(REPO, "yara_amd", "_build",
                                                  "kernels-hip-amdgcn-amd-amdhsa-gfx950.s"))
    ap.add_argument("--tiles", type=int, default=2)
    a = ap.parse_args()
    print(json.dumps(mix(a.asm, a.kernel, a.tiles), indent=1))
