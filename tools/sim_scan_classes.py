"""CPU restatement of the verified-only scan's class decisions (kernels.hip
scan_class_entry): for every 1-byte-key candidate of a golden case, the class
the scan kernel would give it from the eight lane bytes around the key, checked
against the oracle's kept calls (a dead class on a kept call is a bug).
    python tools/sim_scan_classes.py <rules> <case|xs>
"""
import sys, ctypes, numpy as np
import os
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0]=[REPO, os.path.join(REPO, 'tests'), os.path.join(REPO, 'tests', 'golden')]
os.environ['YARA_AMD_LIB']=os.path.join(REPO, 'yara_amd', '_diag', 'libyara_amd.so')
import yara_amd, oracle
from conftest import tables_npz, case_data, golden, ref_tables
L=yara_amd._lib.lib()
rules=sys.argv[1]; case=sys.argv[2]
t=yara_amd.Tables.from_npz(tables_npz(rules), device=0, strings=True)
o=(ctypes.c_uint32*40)()
L.yr_amd__diag_key_classes.argtypes=[ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32)]
print(L.yr_amd__diag_key_classes(t._h, o))
kx_end, byte_keys, nk = o[0], o[1], o[2]
info=o[3:7]; m=o[7:11]; v=o[11:15]; x0=o[15:19]; x1=o[19:23]; minpos=o[23:27]; kx_deep=o[27]; kx_next=o[28]
print("kx_end",kx_end,"keys",[hex(byte_keys>>(8*k)&255) for k in range(nk)],"info",[hex(x) for x in info],"m",[hex(x) for x in m],"v",[hex(x) for x in v],"x0",[hex(x) for x in x0],"x1",[hex(x) for x in x1],"minpos",minpos,"deep",kx_deep,"next",kx_next)
data = oracle.xorshift(64<<20,1) if case=='xs' else case_data(golden()['cases'][case])
n=len(data)
z=np.load(tables_npz(rules))
P,K=oracle.walk_verify(ref_tables(rules), data)
keep=oracle.literal_effect(z,P,K,data)
kept_pos=set(P[keep].tolist())
def excluded(b,x0,x1):
    bs=[(x0>>(8*i))&255 for i in range(4)]+[(x1>>(8*i))&255 for i in range(4)]
    return b in bs
keys=[(byte_keys>>(8*k))&255 for k in range(nk)]
bad=0; dead=0; tot=0
for b in range(n):
    if data[b] not in keys: continue
    tot+=1
    pos=b+1
    k=keys.index(data[b])
    j=b%16
    lane=(b//16)%64
    have=18-j
    w=[int(data[b-2+i]) if 0<=b-2+i<n else 0 for i in range(8)]
    if have<8:
        w=w[:have]
        if kx_next and lane!=63:
            w+= [int(data[b-j+16+i]) if b-j+16+i<n else 0 for i in range(2)]
        have=len(w)
        w=(w+[0]*8)[:8]
    last=min(have,8)-1
    inf=info[k]
    cls=None
    if not inf&1: cls=0
    elif inf&2 and excluded(w[1],x0[k],x1[k]): cls=0
    elif inf&4: cls=2 if pos>=minpos[k] else 0
    else:
        g=ctypes.c_int8(inf>>8&255).value; s0=2+g
        span=inf>>16&15; tmax=inf>>20&3
        end=pos+ctypes.c_int8(inf>>24&255).value
        if end>n: cls=0
        elif s0<0 or s0+span+tmax>last: cls=0
        else:
            W=int.from_bytes(bytes(w),'little')
            hit=any(((W>>(8*(s0+jj)))&m[k]&0xffffffff)==v[k] for jj in range(span+1))
            cls=0 if hit else 1
    if cls==1:
        dead+=1
        if pos in kept_pos: 
            bad+=1
            if bad<5: print("BAD pos",pos,"j",j,"lane",lane,"w",[hex(x) for x in w],"last",last)
print("certain",tot,"dead",dead,"bad",bad)
