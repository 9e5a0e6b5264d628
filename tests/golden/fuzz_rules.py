"""Randomised rule sets + planted buffers (fixture spec for the fuzz parity cases).

``gen(seed)`` writes a small rule file mixing every string form the atom
extractor (atoms.c) and the Aho-Corasick builder (ahocorasick.c) treat
differently: text strings with random modifier combinations (nocase, wide,
ascii wide, xor, xor(a-b), fullword, private, base64), hex strings with ``??``,
nibble wildcards, jumps and alternations, and regexps with classes, dots,
quantifiers and groups.  Strings draw from a small alphabet, so atoms share
prefixes and collide in the trie, and 1-3 byte strings give short atoms.

``buffer(xorshift, seed, size)`` is half alphabet / half random bytes with a
concrete instance of every string planted several times (encoded per its
modifiers) plus near misses that keep the atom and break a later byte, and
instances flush against both ends of the buffer.

Everything is deterministic (CPython ``random`` + the canonical xorshift), so
the GPU box rebuilds the same bytes from the committed spec; make_golden.py
records the stock libyara verify stream for each (seed, size).
"""
import base64
import random

import numpy as np

ALPHA = b"abcdeABxyz01_"


def _wide(b: bytes) -> bytes:
    return bytes(x for c in b for x in (c, 0))


def _flip(b: bytes, r: random.Random) -> bytes:
    return bytes((c ^ 0x20) if chr(c).isalpha() and r.random() < 0.5 else c for c in b)


def _word(r: random.Random, lo: int, hi: int) -> bytes:
    return bytes(r.choice(ALPHA) for _ in range(r.randint(lo, hi)))


# text-string modifier sets libyara accepts (parser.y modifier checks)
MODS = ["", "", "nocase", "wide", "ascii wide", "nocase wide", "nocase ascii wide", "fullword",
        "xor", "xor(1-4)", "wide xor(0x20-0x22)", "ascii wide xor", "private", "fullword wide",
        "base64"]


def _text(r: random.Random):
    short = r.random() < 0.12
    w = _word(r, 1, 3) if short else _word(r, 4, 11)
    mods = r.choice(MODS)
    if "base64" in mods and len(w) < 4:
        w += _word(r, 4 - len(w), 4 - len(w))
    body = w.decode()

    def inst(rr: random.Random) -> bytes:
        b = w
        if "nocase" in mods:
            b = _flip(b, rr)
        if "xor" in mods:
            if "(" in mods:
                a, z = mods[mods.index("(") + 1:mods.index(")")].split("-")
                key = rr.randint(int(a, 0), int(z, 0))
            else:
                key = rr.randint(0, 255)
            b = bytes(c ^ key for c in b)
        if "base64" in mods:
            pad = bytes(rr.choice(ALPHA) for _ in range(rr.randint(0, 2)))
            b = base64.b64encode(pad + b + b"!")
        if "wide" in mods and ("ascii" not in mods or rr.random() < 0.5):
            b = _wide(b)
        if "fullword" in mods and rr.random() < 0.5:
            b = b"." + b + b" "
        return b
    return '"%s"%s' % (body, (" " + mods) if mods else ""), inst


def _hex(r: random.Random):
    toks, gens = [], []
    n = r.randint(2, 7)
    for k in range(n):
        edge = k == 0 or k == n - 1
        t = r.random()
        if edge or t < 0.5:
            v = r.choice(ALPHA) if r.random() < 0.7 else r.getrandbits(8)
            toks.append("%02X" % v)
            gens.append(lambda rr, v=v: bytes([v]))
        elif t < 0.62:
            toks.append("??")
            gens.append(lambda rr: bytes([rr.choice(ALPHA)]))
        elif t < 0.72:
            v = r.choice(ALPHA)
            if r.random() < 0.5:
                toks.append("%X?" % (v >> 4))
                gens.append(lambda rr, v=v: bytes([(v & 0xF0) | rr.getrandbits(4)]))
            else:
                toks.append("?%X" % (v & 0xF))
                gens.append(lambda rr, v=v: bytes([(rr.getrandbits(4) << 4) | (v & 0xF)]))
        elif t < 0.86 and toks and not toks[-1].startswith("["):
            lo = r.randint(0, 3)
            hi = lo + r.randint(0, 5)
            toks.append("[%d-%d]" % (lo, hi))
            gens.append(lambda rr, lo=lo, hi=hi: bytes(rr.choice(ALPHA)
                                                       for _ in range(rr.randint(lo, hi))))
        else:
            alts = [_word(r, 1, 3) for _ in range(r.randint(2, 3))]
            toks.append("( %s )" % " | ".join(" ".join("%02X" % c for c in a) for a in alts))
            gens.append(lambda rr, alts=alts: rr.choice(alts))

    def inst(rr: random.Random) -> bytes:
        return b"".join(g(rr) for g in gens)
    return "{ %s }" % " ".join(toks), inst


def _regex(r: random.Random):
    parts, gens = [], []
    for k in range(r.randint(2, 5)):
        t = r.random()
        c = chr(r.choice(ALPHA))
        if k == 0 or t < 0.4:
            w = _word(r, 1, 3)
            parts.append(w.decode())
            gens.append(lambda rr, w=w: w)
        elif t < 0.55:
            cls = sorted(set(chr(r.choice(ALPHA)) for _ in range(r.randint(2, 4))))
            parts.append("[%s]" % "".join(cls))
            gens.append(lambda rr, cls=cls: rr.choice(cls).encode())
        elif t < 0.65:
            parts.append(".")
            gens.append(lambda rr: bytes([rr.choice(ALPHA)]))
        elif t < 0.8:
            lo = r.randint(0, 2)
            hi = max(1, lo + r.randint(0, 3))   # {0,0} is rejected (re_lexer.l)
            parts.append("%s{%d,%d}" % (c, lo, hi))
            gens.append(lambda rr, c=c, lo=lo, hi=hi: c.encode() * rr.randint(lo, hi))
        elif t < 0.9:
            parts.append("%s+" % c)
            gens.append(lambda rr, c=c: c.encode() * rr.randint(1, 3))
        else:
            alts = [_word(r, 1, 3) for _ in range(2)]
            parts.append("(%s)" % "|".join(a.decode() for a in alts))
            gens.append(lambda rr, alts=alts: rr.choice(alts))
    mods = r.choice(["", "", "nocase", "wide", "ascii wide"])

    def inst(rr: random.Random) -> bytes:
        b = b"".join(g(rr) for g in gens)
        if mods == "nocase":
            b = _flip(b, rr)
        if "wide" in mods and ("ascii" not in mods or rr.random() < 0.5):
            b = _wide(b)
        return b
    return "/%s/%s" % ("".join(parts), (" " + mods) if mods else ""), inst


def _strings(seed: int):
    r = random.Random(seed)
    rules = []
    for i in range(r.randint(2, 5)):
        strs = []
        for j in range(r.randint(2, 9)):
            t = r.random()
            strs.append(_text(r) if t < 0.5 else (_hex(r) if t < 0.8 else _regex(r)))
        cond = r.choice(["any of them", "any of them", "2 of them", "all of them"])
        rules.append((i, strs, cond))
    return rules


def gen(seed: int) -> str:
    out = []
    for i, strs, cond in _strings(seed):
        out.append("rule f%d_%d {\n strings:" % (seed, i))
        out += ["  $s%d = %s" % (j, s) for j, (s, _) in enumerate(strs)]
        out.append(" condition: %s\n}" % cond)
    return "\n".join(out) + "\n"


def _near(b: bytes, rr: random.Random) -> bytes:
    if len(b) < 2:
        return b
    j = rr.randrange(1, len(b))
    return b[:j] + bytes([b[j] ^ 0x41]) + b[j + 1:]


def buffer(xorshift, seed: int, size: int) -> np.ndarray:
    x = xorshift(size, 100 + seed)
    alpha = np.frombuffer(ALPHA, dtype=np.uint8)
    buf = np.where((x & 0x80) != 0, alpha[x % len(ALPHA)], x).astype(np.uint8)
    rr = random.Random(2000 + seed)
    insts = []
    for _, strs, _ in _strings(seed):
        for _, inst in strs:
            insts += [inst(rr) for _ in range(3)] + [_near(inst(rr), rr) for _ in range(2)]
    insts = [b for b in insts if 0 < len(b) < size]
    for b in insts:
        pos = rr.randrange(0, size - len(b) + 1)
        buf[pos:pos + len(b)] = np.frombuffer(b, dtype=np.uint8)
    if insts:   # flush against both ends: the first / last window of the scan
        head, tail = insts[0], insts[-1]
        buf[:len(head)] = np.frombuffer(head, dtype=np.uint8)
        buf[size - len(tail):] = np.frombuffer(tail, dtype=np.uint8)
    return buf


if __name__ == "__main__":
    import sys
    print(gen(int(sys.argv[1])), end="")
