"""Per-tile instruction budget of a scan-kernel variant, read from its ISA.

Builds nothing: reads the assembly `make -C yara_amd/csrc asm` leaves in
yara_amd/_build/kernels-hip-amdgcn-amd-amdhsa-gfx950.s and classifies the
instructions of named basic-block ranges of one kernel (VALU by issue class:
VOP2 / VOP3-class incl. DPP and SDWA, which issue at half rate on gfx950 --
DESIGN.md §5; SALU; LDS; VMEM; waits).  The hot path of
scan_segments_kernel<0> is located by its markers: the tile step starts at the
block holding the tile's buffer_load (stage 1), the drain at the block holding
the ring entry's three ds_read, and so on (see PATHS).

    python tools/isa_budget.py [--kernel 0] [--json]
"""
import argparse
import json
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASM = os.environ.get("YAMD_ASM") or os.path.join(REPO, "yara_amd", "_build", "kernels-hip-amdgcn-amd-amdhsa-gfx950.s")
HALF = ("v_alignbyte_b32", "v_perm_b32", "v_bitop3_b32", "v_mad_u32_u24", "v_lshl_add_u32",
        "v_add3_u32", "v_mbcnt_lo_u32_b32", "v_mbcnt_hi_u32_b32", "v_readlane_b32",
        "v_readfirstlane_b32", "v_writelane_b32", "v_lshl_add_u64", "v_bfe_u32", "v_lshl_or_b32",
        "v_and_or_b32", "v_or3_b32", "v_xad_u32", "v_cndmask_b32_e64", "v_lshrrev_b64",
        "v_dot4_u32_u8")


def kind(line):
    t = line.split()
    op = t[0]
    if op.startswith("v_"):
        if "_dpp" in op or " row_" in line or "wave_" in line:
            return "valu_dpp"
        if "_sdwa" in op:
            return "valu_sdwa"
        if op in HALF or op.endswith("_e64"):
            return "valu_vop3"
        return "valu_vop2"
    if op.startswith(("s_waitcnt", "s_nop")):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_")):
        return "vmem"
    return None


def blocks(kernel):
    src = open(ASM).read().split("\n")
    name = "_ZN4yamd20scan_segments_kernelILi%dEEEvNS_10ScanParamsE" % kernel
    start = next(i for i, l in enumerate(src) if l.startswith(name + ":"))
    end = next(i for i in range(start, len(src)) if src[i].startswith(".Lfunc_end"))
    out, cur = [], {"label": "entry", "insts": []}
    for l in src[start + 1:end]:
        t = l.strip()
        m = re.match(r"^(\.LBB\d+_\d+):", t) or re.match(r"^; (%bb\.\d+):", t)
        if m:
            out.append(cur)
            cur = {"label": m.group(1), "insts": []}
            continue
        if not t or t.startswith((";", ".")):
            continue
        cur["insts"].append(t)
    out.append(cur)
    return out


def count(insts):
    c = {}
    for t in insts:
        k = kind(t)
        if k:
            c[k] = c.get(k, 0) + 1
    c["valu"] = sum(v for k, v in c.items() if k.startswith("valu_"))
    # VOP2-equivalent issue slots: VOP3-class, DPP and SDWA forms at half rate
    c["valu_vop2_equiv"] = c.get("valu_vop2", 0) + 2 * (c["valu"] - c.get("valu_vop2", 0))
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", type=int, default=0)
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    bb = blocks(a.kernel)
    # the main loop's two tile steps start at the blocks holding a tile load
    # (buffer_load_dwordx4 ... offen nt) followed by stage 1's ds_read_b64s
    loads = [i for i, b in enumerate(bb) if any(t.startswith("buffer_load_dwordx4") for t in b["insts"])
             and sum(t.startswith("ds_read_b64") for t in b["insts"]) >= 8]
    res = {"kernel": "scan_segments_kernel<%d>" % a.kernel, "asm": os.path.relpath(ASM, REPO)}
    if loads:
        st = bb[loads[0]]
        res["stage1_block"] = {"label": st["label"], **count(st["insts"])}
    # the drain's re-test: the block that reads a ring entry (three 8-byte
    # LDS reads of one entry) and then 8 filter blocks
    for i, b in enumerate(bb):
        n64 = sum(t.startswith(("ds_read_b64", "ds_read2_b64")) for t in b["insts"])
        if n64 >= 9 and not any(t.startswith("buffer_load") for t in b["insts"]):
            res["drain_retest_block"] = {"label": b["label"], **count(b["insts"])}
            break
    res["whole_kernel"] = count([t for b in bb for t in b["insts"]])
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
