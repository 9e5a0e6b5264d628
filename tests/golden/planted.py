"""Planted functional buffers (fixture spec, SURVEY.md §8d "planted" variant).

A planted buffer is xorshift64 random bytes (seed 3) with a concrete instance of
every generated string copied in twice at positions drawn from
``random.Random(seed)``; nocase strings get a random case flip on the second
copy.  Unlike the pure-random perf buffers these produce real matches, so the
verifier (scan.c / re.c) and the rule conditions are exercised end to end.

Everything here is deterministic (CPython ``random`` + the canonical xorshift),
so the same bytes are rebuilt on the GPU box from the committed specs.
"""
import random
import re

import numpy as np

_TOKEN = re.compile(r"\?\?|[0-9A-Fa-f]\?|\?[0-9A-Fa-f]|[0-9A-Fa-f]{2}|\[\d+-\d+\]")


def _instance_hex(body: str, r: random.Random) -> bytes:
    out = bytearray()
    for tok in _TOKEN.findall(body):
        if tok == "??":
            out.append(r.getrandbits(8))
        elif tok.startswith("["):
            lo, hi = map(int, tok[1:-1].split("-"))
            out.extend(r.getrandbits(8) for _ in range(r.randint(lo, hi)))
        elif tok.endswith("?"):
            out.append((int(tok[0], 16) << 4) | r.getrandbits(4))
        elif tok.startswith("?"):
            out.append((r.getrandbits(4) << 4) | int(tok[1], 16))
        else:
            out.append(int(tok, 16))
    return bytes(out)


def string_instances(rules_text: str, seed: int = 7):
    """One concrete byte instance per string of a generated rule file.

    Returns a list of (bytes, nocase) in declaration order.
    """
    r = random.Random(seed)
    out = []
    for line in rules_text.splitlines():
        line = line.strip()
        if not line.startswith("$"):
            continue
        _, rhs = line.split("=", 1)
        rhs = rhs.strip()
        if rhs.startswith("{"):
            out.append((_instance_hex(rhs[1:rhs.rindex("}")], r), False))
        else:
            lit = rhs[1:rhs.rindex('"')]
            out.append((lit.encode(), rhs.endswith("nocase")))
    return out


def _flip_case(b: bytes, r: random.Random) -> bytes:
    return bytes((c ^ 0x20) if (65 <= c <= 90 or 97 <= c <= 122) and r.random() < 0.5 else c
                 for c in b)


def planted_buffer(xorshift, rules_text: str, size: int, seed: int = 3) -> np.ndarray:
    """xorshift(size, seed) with every string instance planted twice."""
    buf = xorshift(size, seed).copy()
    r = random.Random(1000 + seed)
    for data, nocase in string_instances(rules_text):
        for copy in range(2):
            inst = _flip_case(data, r) if (nocase and copy == 1) else data
            pos = r.randrange(0, size - len(inst))
            buf[pos:pos + len(inst)] = np.frombuffer(inst, dtype=np.uint8)
    return buf


def boundary_buffer(xorshift, atoms, size: int, period: int, seed: int = 11) -> np.ndarray:
    """Random bytes with atoms planted so they END exactly at multiples of
    ``period`` (and one byte either side): the adversarial slice/shard-edge case
    of SURVEY.md Appendix A's parity-trap list."""
    buf = xorshift(size, seed).copy()
    r = random.Random(seed)
    k = 0
    for end in range(period, size, period):
        a = atoms[k % len(atoms)]
        k += 1
        e = end + r.choice((-1, 0, 0, 1))
        if e - len(a) >= 0 and e <= size:
            buf[e - len(a):e] = np.frombuffer(a, dtype=np.uint8)
    return buf


# --- literal-variety buffer (tests/golden/rules/lit.yar) ---------------------
# Every literal form the on-device pre-verification restates (scan.c:62-255,
# 887-990) is planted as a match and as near misses that pass the atom but fail
# the comparison: ascii / wide / nocase / xor (narrow and wide, several keys) /
# fixed offset / fullword / base64 / hex with wildcards and jumps.
LIT_WORDS = [b"HelloWorld", b"xyzzy1234", b"ab", b"Quartz", b"WideString", b"AsciiAndWide",
             b"CaseLess", b"NoCaseWide", b"zz", b"XorMe!", b"XorWide", b"XorRange",
             b"FixedHere", b"word", b"secretstr"]


def _wide(b: bytes) -> bytes:
    return bytes(x for c in b for x in (c, 0))


def _near(b: bytes, r: random.Random) -> bytes:
    """Same first 4 bytes (atom still hits), one later byte changed."""
    if len(b) <= 4:
        return b[:-1] + bytes([b[-1] ^ 0x01])
    j = r.randrange(4, len(b))
    return b[:j] + bytes([b[j] ^ 0x5A]) + b[j + 1:]


def lit_buffer(xorshift, size: int, seed: int = 13) -> np.ndarray:
    import base64
    buf = xorshift(size, seed).copy()
    r = random.Random(seed)
    pieces = []
    for w in LIT_WORDS:
        pieces += [w, _wide(w), _flip_case(w, r), _near(w, r), _wide(_near(w, r))]
        for key in (0x01, 0x10, 0x5A, 0xFF):
            pieces.append(bytes(c ^ key for c in w))
            pieces.append(bytes(c ^ key for c in _wide(w)))
            pieces.append(bytes(c ^ key for c in _near(w, r)))
    pieces += [b" word ", b"swordfish", b"word.", b"(word)", b"words"]
    for t in (b"base64text", b"xbase64text", b"xxbase64text"):
        pieces.append(base64.b64encode(t))
    pieces += [bytes.fromhex("414243444546"), bytes.fromhex("4142434445FF"),
               bytes.fromhex("6162AA6465"), bytes.fromhex("6162AA6466"),
               bytes.fromhex("313233AABB3738"), bytes.fromhex("313233AABBCCDD3738"),
               bytes.fromhex("313233AA3738")]
    for p in pieces:
        for _ in range(2):
            pos = r.randrange(0, size - len(p))
            buf[pos:pos + len(p)] = np.frombuffer(p, dtype=np.uint8)
    fixed = b"FixedHere"
    if size > 8192:
        buf[4096:4096 + len(fixed)] = np.frombuffer(fixed, dtype=np.uint8)
        buf[6000:6000 + len(fixed)] = np.frombuffer(fixed, dtype=np.uint8)
    return buf


# --- hex-with-jumps buffer (tests/golden/rules/hex.yar) ----------------------
# Instances and near misses of every hex string (the fast-exec programs of
# re.c:2150-2391): jumps at their bounds and one past, masked nibbles, ~XX,
# atoms near the block start/end (backward / forward limits), a long jump.
def hex_buffer(xorshift, size: int, seed: int = 17) -> np.ndarray:
    buf = xorshift(size, seed).copy()
    r = random.Random(seed)
    H = bytes.fromhex
    pieces = []
    for gap in range(1, 9):
        pieces.append(H("4D5A01025045") + bytes(gap) + H("1122"))
    for g1 in range(0, 5):
        for g2 in range(0, 4):
            pieces.append(H("AABBCCDD") + b"\x77" * g1 + H("EE") + b"\x66" * g2 + H("FF01"))
    for g in (3, 4, 5):
        pieces.append(H("1020") + bytes(g) + H("30405060"))
    for g in (0, 1, 5, 10, 11):
        pieces.append(H("71727374A57B") + b"\x33" * g + H("75"))
        pieces.append(H("71727374A67B") + b"\x33" * g + H("75"))   # masked miss
    for x in (0x02, 0x03, 0x04):
        pieces.append(H("0102") + bytes([x]) + H("040506"))
    for a, b_, c in ((1, 1, 1), (2, 2, 2), (1, 2, 3), (3, 1, 1)):
        pieces.append(H("81828384") + bytes(a) + H("85") + bytes(b_) + H("86") + bytes(c) + H("87"))
    for g in (0, 1, 4, 5):
        pieces.append(H("9A9B") + b"\x44" * g + H("C1C2C3C4"))
        pieces.append(H("9A9C") + b"\x44" * g + H("C1C2C3C4"))      # backward miss
    for g in (1, 2, 3, 4):
        pieces.append(H("E100E3") + b"\x55" * g + H("F1F2F3F4F5"))
    pieces += [H("5A6B7C8D91929394"), H("5A6B7C9D91929394"), H("5A6B7C8D91929395")]
    for g in (99, 100, 2999, 3000, 3001):
        pieces.append(H("31415926") + bytes(g) + H("53589793"))
    for p in pieces:
        for _ in range(2):
            pos = r.randrange(16, size - len(p) - 16)
            buf[pos:pos + len(p)] = np.frombuffer(p, dtype=np.uint8)
    # block-edge cases: a string whose atom sits right at the start / end
    edge = H("C1C2C3C4")
    buf[0:4] = np.frombuffer(edge, np.uint8)                  # no room for the prefix
    tail = H("4D5A01025045") + bytes(2) + H("11")           # truncated at the end
    buf[size - len(tail):] = np.frombuffer(tail, np.uint8)
    return buf


# --- regexp buffer (tests/golden/rules/rx.yar) --------------------------------
# Matches and near misses of yr_re_exec programs (re.c:1693): classes, optional
# groups, alternation, bounded / unbounded repeats, word boundaries, nocase,
# wide, dot-all, and hex strings with alternatives (not fast-exec programs).
def rx_buffer(xorshift, size: int, seed: int = 19) -> np.ndarray:
    buf = xorshift(size, seed).copy()
    r = random.Random(seed)
    H = bytes.fromhex
    pieces = [b"http://abc.com", b"https://example12.com", b"http://ab.com", b"https://abc.org",
              b"Content-Type: text/html", b"CONTENT-TYPE: Application/JSON", b"Content-Type: 1/2",
              b"username=alice_01", b"username_id=bob42", b"username=ab", b"username_id=",
              b" password ", b"xpassword ", b"(password)", b"passwords",
              b"GET /index.php?id=42", b"GET /index.php?id=", b"GET /Index.php?id=1",
              b"abcde12vwxyz", b"abcde\n\n\nvwxyz", b"abcde1vwxyz", b"abcde123456vwxyz",
              b"cathouse", b"doghouse", b"birdhouse", b"cowhouse", b"Qx1234Zq!", b"Qx12\n4Zq!",
              b"Qx1Zq!", b"Qx123456789Zq!"]
    for w in (b" password ", b"password", b"xpasswordx"):
        pieces.append(bytes(x for c in w for x in (c, 0)))
    pieces += [H("4D5A9000030102FFFF"), H("4D5A5000030102030405FFFF"), H("4D5A9100030102FFFF"),
               H("4D5A900003FFFF"), H("E8010203045BC3"), H("E8010203045DC3"), H("E8010203045CC3"),
               H("1122334455BB"), H("112233446677BB"), H("112233448899AABB"),
               H("112233446699BB")]
    for p in pieces:
        for _ in range(3):
            pos = r.randrange(16, size - len(p) - 16)
            buf[pos:pos + len(p)] = np.frombuffer(p, dtype=np.uint8)
    # an atom right at the block start and a match cut by the block end
    head = b"cathouse"
    buf[0:len(head)] = np.frombuffer(head, np.uint8)
    tail = b"https://abcd.co"
    buf[size - len(tail):] = np.frombuffer(tail, np.uint8)
    return buf
