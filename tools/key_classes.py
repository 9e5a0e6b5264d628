"""The 1-byte keys' class records (scanner.cpp key_classes, ScanParams::kc)
of golden tables, decoded (diagnostic build's yr_amd__diag_key_classes).
GPU box:  python tools/key_classes.py rx fuzz0 ...
"""
import ctypes, json, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ["YARA_AMD_LIB"] = os.path.join(REPO, "yara_amd", "_diag", "libyara_amd.so")
import yara_amd
L = yara_amd._lib.lib()
g = L.yr_amd__diag_key_classes
g.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32)]
s8 = lambda x: x - 256 if x >= 128 else x
for name in sys.argv[1:]:
    t = yara_amd.Tables.from_npz(os.path.join(REPO, "tests", "golden", "tables", name + ".npz"), device=0, strings=True)
    o = (ctypes.c_uint32 * 40)()
    g(t._h, o)
    keys = []
    for k in range(o[2]):
        info, mp = o[3 + k], o[23 + k]
        keys.append({"key": hex(o[1] >> (8 * k) & 255), "info": hex(info), "class": bool(info & 1),
                     "excl": bool(info & 2), "kept": bool(info & 4), "bguard": bool(info & 8),
                     "rs": s8(info >> 8 & 255), "span": info >> 16 & 15, "tmax": info >> 20 & 3,
                     "end": s8(info >> 24 & 255), "m": hex(o[7 + k]), "v": hex(o[11 + k]),
                     "x": [hex(o[15 + k]), hex(o[19 + k])], "min_pos": mp, "bm": hex(o[32 + k]),
                     "bv": hex(o[36 + k])})
    print(json.dumps({"rules": name, "kx_end": o[0], "kx_deep": o[27], "kx_next": o[28], "keys": keys}), flush=True)
