"""Candidates of a 1 GiB scan that the byte-key drain classified (kernels.hip
key_class: dead or kept), counted through the diagnostic build's
yr_amd__diag_dead_count.  GPU box:  python tools/dead_count.py
"""
import ctypes, os, sys
sys.path.insert(0, os.getcwd())
os.environ["YARA_AMD_LIB"] = os.path.join(os.getcwd(), "yara_amd/_diag/libyara_amd.so")
import torch, yara_amd
from yara_amd import _lib
L = _lib.lib(); f = L.yr_amd__diag_dead_count; f.restype = ctypes.c_int64; f.argtypes = [ctypes.c_void_p]
for rules, gib in (("rx", 1), ("fuzz0", 1)):
    n = gib << 30
    buf = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    yara_amd.fill_xorshift64(buf.data_ptr(), n, 1)
    t = yara_amd.Tables.from_npz(os.path.join("tests/golden/tables", rules + ".npz"), device=0, strings=True)
    sc = yara_amd.Scanner(t)
    for _ in range(2):
        sc.scan_device(buf.data_ptr(), n); _, cnt, _ = sc.device_result()
        print(rules, "candidates", cnt, "dead", f(sc._h), flush=True)

# the key classes of every golden table with 1-byte keys (yr_amd__diag_key_classes)
g = L.yr_amd__diag_key_classes; g.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32)]
for name in sorted(os.listdir("tests/golden/tables")):
    t = yara_amd.Tables.from_npz(os.path.join("tests/golden/tables", name), device=0, strings=True)
    o = (ctypes.c_uint32 * 40)()
    g(t._h, o)
    if o[2]:
        print(name[:-4], "kx_end", o[0], "keys", [hex(o[1] >> (8 * k) & 255) for k in range(o[2])],
              "info", [hex(x) for x in o[3:7]], "m", [hex(x) for x in o[7:11]], "v", [hex(x) for x in o[11:15]], flush=True)
