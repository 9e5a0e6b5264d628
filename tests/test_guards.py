"""Program guards of the on-device pre-verification (verify.h DevGuard), CPU side.

The host compiles, per regexp program, 4 positions the program must consume with
their byte tests (scanner.cpp fast_guard / general_guard); the verify kernel
drops a call whose input fails them before interpreting the program.  That is
sound only if every input the program matches passes its guard.  Checked here
through the library's guard compiler (yr_amd__program_guard, a diagnostic
export) against a restatement of yr_re_fast_exec's linear programs
(re.c:2150-2391: LITERAL, MASKED_LITERAL, ANY, the NOT forms, REPEAT_ANY_UNGREEDY,
MATCH) on random programs and inputs built to match them, and on hand-written
yr_re_exec programs (JUMPs, zero-width assertions, SPLIT, CLASS, nocase).
"""
import ctypes
import random

import pytest

from yara_amd import _lib

ANY, LIT, MASKED, CLASS, MATCH, NOTLIT, MASKEDNOT = 0xA0, 0xA2, 0xA4, 0xA5, 0xAD, 0xAE, 0xAF
WORDB, REPANYG, REPANY, SPLITA, JUMP = 0xB2, 0xB4, 0xB5, 0xC0, 0xC2


def guard(code, skip=0, backwards=False, general=False, nocase=False):
    L = _lib.lib()
    f = L.yr_amd__program_guard
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_int,
                  ctypes.c_int] + [ctypes.POINTER(ctypes.c_uint32)] * 3
    m, v, bs = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    r = f(bytes(code), len(code), skip, int(backwards), int(general), int(nocase),
          ctypes.byref(m), ctypes.byref(v), ctypes.byref(bs))
    assert r in (0, 1)
    return (m.value, v.value, bs.value) if r else None


def guard_passes(g, x, backwards):
    """The kernel's test (verify.hip guard_ok) on x = the input bytes in the
    order the program reads them; True when the bytes are not all there."""
    m, v, bs = g
    base, span = bs & 15, bs >> 4
    if base + span + 4 > len(x):
        return True
    for j in range(span + 1):
        ok = True
        for t in range(4):
            sh = 8 * (3 - t if backwards else t)
            mt, vt = (m >> sh) & 0xFF, (v >> sh) & 0xFF
            if mt and (x[base + j + t] & mt) != vt:
                ok = False
        if ok:
            return True
    return False


def fast_matches(code, x):
    """Can the linear fast program reach MATCH on x (re.c:2150-2391, positions as
    a set; every consuming opcode needs b < len(x))?"""
    live, ip, n = {0}, 0, len(x)
    while live:
        op = code[ip]
        if op == MATCH:
            return True
        if op == REPANY:
            mn = code[ip + 1] | code[ip + 2] << 8
            mx = code[ip + 3] | code[ip + 4] << 8
            live = {b + k for b in live for k in range(mn, mx + 1) if k == mn or b + k < n}
            ip += 5
            continue
        if op == ANY:
            test, size = (lambda c: True), 1
        elif op in (LIT, NOTLIT):
            val = code[ip + 1]
            test, size = ((lambda c, val=val: c == val) if op == LIT else (lambda c, val=val: c != val)), 2
        else:
            val, mask = code[ip + 1], code[ip + 2]
            test = ((lambda c, val=val, mask=mask: (c & mask) == val) if op == MASKED
                    else (lambda c, val=val, mask=mask: (c & mask) != val))
            size = 3
        live = {b + 1 for b in live if b < n and test(x[b])}
        ip += size
    return False


def random_fast_program(r):
    """Program and one input it matches."""
    code, inp = [], []
    repeats = 0
    for _ in range(r.randint(1, 9)):
        k = r.random()
        if k < 0.45:
            c = r.randrange(256)
            code += [LIT, c]
            inp.append(c)
        elif k < 0.6:
            mask = r.choice([0xF0, 0x0F, 0xFE, 0x3C])
            c = r.randrange(256)
            code += [MASKED, c & mask, mask]
            inp.append(c)
        elif k < 0.75:
            code.append(ANY)
            inp.append(r.randrange(256))
        elif k < 0.82:
            c = r.randrange(256)
            code += [NOTLIT, c]
            inp.append((c + 1 + r.randrange(255)) % 256)
        elif repeats < 2:
            mn = r.randint(0, 3)
            mx = mn + r.randint(0, 9)
            code += [REPANY, mn & 255, mn >> 8, mx & 255, mx >> 8]
            inp += [r.randrange(256) for _ in range(r.randint(mn, mx))]
            repeats += 1
    code.append(MATCH)
    return bytes(code), bytes(inp)


def as_greedy(code):
    """The program with its REPEAT_ANY_UNGREEDY opcodes made greedy."""
    out, ip = bytearray(code), 0
    size = {ANY: 1, LIT: 2, NOTLIT: 2, MASKED: 3, MASKEDNOT: 3, REPANY: 5, MATCH: 1}
    while ip < len(code):
        if code[ip] == REPANY:
            out[ip] = REPANYG
        ip += size[code[ip]]
    return bytes(out)


@pytest.mark.parametrize("general", [False, True], ids=["fast", "general"])
@pytest.mark.parametrize("seed", range(8))
def test_fast_guards_never_reject_a_match(seed, general):
    """Also as yr_re_exec programs (general): on a linear program they accept a
    subset of what the fast model accepts (their ANY / REPEAT_ANY refuse 0x0A
    without DOT_ALL), so a guard that passes every fast match is sound for
    them; REPEAT_ANY_GREEDY enumerates the same counts."""
    r = random.Random(seed)
    guarded = rejected = 0
    for _ in range(400):
        code, inp = random_fast_program(r)
        backwards = r.random() < 0.5
        skip = r.randint(0, 4)
        g = guard(code, skip=skip, backwards=backwards, general=general)
        if general and r.random() < 0.5:
            greedy = as_greedy(code)
            assert guard(greedy, skip=skip, backwards=backwards, general=True) == g
        if g is None:
            continue
        guarded += 1
        tail = bytes(r.randrange(256) for _ in range(r.randint(0, 12)))
        x = inp + tail
        assert fast_matches(code, x)
        assert guard_passes(g, x, backwards), (code.hex(), x.hex(), g)
        for _ in range(20):   # mutated inputs: whenever the program matches, so does the guard
            y = bytearray(x)
            for _ in range(r.randint(1, 3)):
                y[r.randrange(len(y))] = r.randrange(256)
            if fast_matches(code, bytes(y)):
                assert guard_passes(g, bytes(y), backwards), (code.hex(), bytes(y).hex(), g)
            elif not guard_passes(g, bytes(y), backwards):
                rejected += 1
    assert guarded > 100 and rejected > 100


def test_fast_guard_shapes():
    # atom 36 9B 09 94 then ?? AE 28 [1-8] A3: the first window with the most
    # tested bits past the atom (positions 3..6: 94 ?? AE 28)
    code = bytes([LIT, 0x36, LIT, 0x9B, LIT, 0x09, LIT, 0x94, ANY, LIT, 0xAE, LIT, 0x28,
                  REPANY, 1, 0, 8, 0, LIT, 0xA3, MATCH])
    m, v, bs = guard(code, skip=4)
    assert bs == 3 and m == 0xFFFF00FF and v == 0x28AE0094
    # backward program REPEAT_ANY {1,8} then 5C ?? 57 B7: after the repeat,
    # span 7, memory order (byte 3 = the first byte read)
    code = bytes([REPANY, 1, 0, 8, 0, LIT, 0x5C, ANY, LIT, 0x57, LIT, 0xB7, LIT, 0x3B, MATCH])
    m, v, bs = guard(code, backwards=True)
    assert bs == 1 | 7 << 4 and m == 0xFF00FFFF and v == 0x5C0057B7
    # the atom alone: nothing to test
    assert guard(bytes([LIT, 1, LIT, 2, LIT, 3, MATCH]), skip=3) is None


def test_general_guard_follows_jumps_and_stops_at_splits():
    # { E8 ?? ?? ?? ?? ( 5B | 5D ) C3 } from the atom 5B: 5B, JUMP over 5D, C3
    fwd = bytes([LIT, 0x5B, JUMP, 5, 0, LIT, 0x5D, LIT, 0xC3, MATCH])
    assert guard(fwd, skip=1, general=True) == (0x0000FFFF, 0x0000C35B, 0)
    # its backward program: JUMP over 5D, four ANY, E8 (memory order: byte 0)
    bwd = bytes([JUMP, 5, 0, LIT, 0x5D, ANY, ANY, ANY, ANY, LIT, 0xE8, MATCH])
    assert guard(bwd, backwards=True, general=True) == (0x000000FF, 0x000000E8, 1)
    # zero-width assertions consume nothing; CLASS consumes one untested byte
    cls = bytes([CLASS, 0] + [0xFF] * 32)
    prog = bytes([WORDB]) + cls + bytes([LIT, 0x41, LIT, 0x42, MATCH])
    assert guard(prog, general=True) == (0x00FFFF00, 0x00424100, 0)
    # past the first REPEAT_ANY: { 5F ?? 62 61 ( 31 | ... ) [0-4] 3E }-like forward
    # program from the atom 5F (JUMP over dead code): 3E at distance 1 + j, j <= 4
    fwd = bytes([LIT, 0x5F, JUMP, 9, 0, LIT, 0x61, LIT, 0x62, LIT, 0x31,
                 REPANY, 0, 0, 4, 0, LIT, 0x3E, MATCH])
    assert guard(fwd, skip=1, general=True) == (0x000000FF, 0x0000003E, 1 | 4 << 4)
    assert guard(bytes([REPANYG]) + fwd[12:], general=True) == (0xFF, 0x3E, 0 | 4 << 4)
    # a second repeat ends the tail
    two = bytes([LIT, 1, REPANY, 0, 0, 2, 0, REPANY, 1, 0, 3, 0, LIT, 2, MATCH])
    assert guard(two, skip=1, general=True) is None
    # a SPLIT first: more than one fiber, no guard
    assert guard(bytes([SPLITA, 0, 6, 0, LIT, 0x41, LIT, 0x42, MATCH]), general=True) is None
    # nocase literals compare through the host's case folding: untested
    assert guard(bytes([LIT, 0x41, LIT, 0x42, MATCH]), general=True, nocase=True) is None


# --- fiber safety of yr_re_exec forward programs (scanner.cpp re_fiber_safe) --
REPSTARTG, REPENDG = 0xC3, 0xC4


def fiber_safe(code):
    L = _lib.lib()
    f = L.yr_amd__re_fiber_safe
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_char_p, ctypes.c_uint32]
    r = f(bytes(code), len(code))
    assert r in (0, 1)
    return bool(r)


def test_fiber_safe_bound():
    """A forward program may let a key class test the call's backward guard
    first only if yr_re_exec cannot end in ERROR_TOO_MANY_RE_FIBERS
    (re.c:1228-1229): no REPEAT_START / REPEAT_END (fiber stacks stay empty),
    and ops x (largest REPEAT_ANY max + 2) x (SPLITs + REPEAT_ANYs + 2) below
    RE_MAX_FIBERS = 1024 (limits.h:168)."""
    # fuzz0's key `_` (golden tables): LIT 5F, JUMP +9, dead LITs, REPEAT_ANY {0, 4}, LIT 3E, MATCH
    fuzz0 = [LIT, 0x5F, JUMP, 9, 0, LIT, 0x61, LIT, 0x62, LIT, 0x31, REPANY, 0, 0, 4, 0, LIT, 0x3E, MATCH]
    assert fiber_safe(fuzz0)                      # 8 ops x 6 x 3 = 144
    assert fiber_safe([LIT, 0x41, MATCH])
    # a counted loop: its counter stacks make fibers distinct beyond (ip, rc)
    assert not fiber_safe([REPSTARTG, 2, 0, 5, 0, 9, 0, 0, 0, LIT, 0x41,
                           REPENDG, 2, 0, 5, 0, 0xF7, 0xFF, 0xFF, 0xFF, MATCH])
    # a wide jump: 3 ops x (1000 + 2) x 3 > 1024
    assert not fiber_safe([LIT, 0x41, REPANY, 0, 0, 0xE8, 0x03, LIT, 0x42, MATCH])
    # many ops: 200 literals x (4 + 2) x 3
    assert not fiber_safe([LIT, 0x41] * 199 + [REPANY, 0, 0, 4, 0, MATCH])
    # unknown opcode or a truncated instruction: not provably safe
    assert not fiber_safe([0x99, MATCH])
    assert not fiber_safe([LIT])
