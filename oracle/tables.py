"""Reader for the reference-table dumps written by ``oracle/refdump tables``.

Test infrastructure (oracle): parses T (YR_AC_TRANSITION[], ahocorasick.h:37-50),
M (ac_match_table) and the YR_AC_MATCH pool exactly as libyara exposes them
in YR_RULES (rules.c:356-363), plus the YR_STRING records.
"""
import struct
from dataclasses import dataclass, field

import numpy as np


@dataclass
class RefTables:
    T: np.ndarray                 # uint32[n_slots]
    M: np.ndarray                 # uint32[n_slots], 1-based pool index, 0 = none
    pool_next: np.ndarray         # uint32[n_pool], 1-based next index, 0 = end
    pool_string: np.ndarray       # uint32[n_pool]
    pool_backtrack: np.ndarray    # uint16[n_pool]
    strings: list = field(default_factory=list)
    n_rules: int = 0
    # v2: fast-exec RE programs per pool entry (kind 1) -- re.c:2150
    re_kind: np.ndarray = None    # uint8[n_pool]
    re_fwd: list = None           # bytes per pool entry (b"" if none)
    re_bwd: list = None


def read_tables(path: str) -> RefTables:
    with open(path, "rb") as f:
        buf = f.read()
    assert buf[:4] == b"YRTB", "not a refdump table file"
    ver, ns, npool, nstr, nrules = struct.unpack_from("<5I", buf, 4)
    assert ver in (1, 2)
    off = 24
    T = np.frombuffer(buf, dtype="<u4", count=ns, offset=off).copy(); off += 4 * ns
    M = np.frombuffer(buf, dtype="<u4", count=ns, offset=off).copy(); off += 4 * ns
    pool = np.frombuffer(buf, dtype="<u4", count=3 * npool, offset=off).reshape(npool, 3)
    off += 12 * npool
    strings = []
    for _ in range(nstr):
        flags, rule_idx, length, chained, gmin, gmax = struct.unpack_from("<6I", buf, off)
        (fixed,) = struct.unpack_from("<q", buf, off + 24)
        off += 32
        data = buf[off:off + length]
        off += length + ((4 - (length & 3)) & 3)
        strings.append(dict(flags=flags, rule_idx=rule_idx, length=length,
                            chained_to=None if chained == 0xFFFFFFFF else chained,
                            gap_min=gmin, gap_max=gmax, fixed_offset=fixed, data=data))
    kinds, fwd, bwd = np.zeros(npool, np.uint8), [], []
    if ver >= 2:
        for k in range(npool):
            kind, fl, bl = struct.unpack_from("<3I", buf, off)
            off += 12
            kinds[k] = kind
            fwd.append(buf[off:off + fl])
            bwd.append(buf[off + fl:off + fl + bl])
            off += fl + bl + ((4 - ((fl + bl) & 3)) & 3)
    assert off == len(buf)
    return RefTables(T, M, pool[:, 0].copy(), pool[:, 1].copy(),
                     pool[:, 2].astype(np.uint16), strings, nrules, kinds, fwd, bwd)
