"""The CPU restatement (oracle/) pinned against the reference.

1. The known-answer values of the reference's own test/test_bra_encoders.cpp (hard-coded here).
2. Every golden vector in tests/golden/golden.npz (produced by the reference encoders compiled from
   /root/reference, see tests/golden/make_golden.py), stage by stage.
3. When oracle/_ref/libbraref.so is present: seeded random cross-checks against the reference.
"""
import os
import random

import pytest

from oracle import Reference, have_ref


# ---- 1. reference KATs (test/test_bra_encoders.cpp:23-402) --------------------------------
def test_kat_rle(orc):
    assert orc.rle_encode(b"A" * 10) == bytes([(-9) & 0xFF, ord("A")])  # :23-50
    assert orc.rle_encode(b"AAAAABBBCD") == bytes([(-4) & 0xFF, 65, (-2) & 0xFF, 66, 1, 67, 68])  # :52-90
    assert len(orc.rle_encode(b"ABCDEFGH")) == 9  # :92-114
    for s in (b"A" * 10, b"AAAAABBBCD", b"ABCDEFGH"):
        assert orc.rle_decode(orc.rle_encode(s)) == s


def test_kat_bwt(orc):
    assert orc.bwt_encode(b"BANANA") == (b"NNBAAA", 3)  # :134-141
    fox = b"The quick brown fox jumps over the lazy dog."
    assert orc.bwt_encode(fox) == (b"kynxeserg.l i hhv otTu c uwd rfm ebp qjoooza", 9)  # :143-150
    assert orc.bwt_decode(b"NNBAAA", 3) == b"BANANA"


def test_kat_mtf(orc):
    assert orc.mtf_encode(b"BANANA") == bytes([66, 66, 78, 1, 1, 1])  # :152-170
    assert orc.mtf_decode(bytes([0x4E, 0, 0x43, 0x43, 0, 0])) == b"NNBAAA"  # :199-218


def test_kat_huffman(orc):
    lens, osz, esz, pay = orc.huffman_encode(b"BANANA")  # :262-288
    assert (osz, esz) == (6, 2) and lens[0] == 0
    assert (lens[ord("A")], lens[ord("B")], lens[ord("N")]) == (1, 2, 2)
    assert pay == bytes([155, 0])
    lens, osz, esz, pay = orc.huffman_encode(b"AAAAA")  # :290-333
    assert (osz, esz, lens[ord("A")], pay) == (5, 1, 1, b"\0")
    assert orc.huffman_encode(b"") is None  # :358-365
    mtf = bytes([0x4E, 0, 0x43, 0x43, 0, 0])  # :335-356
    lens, osz, esz, pay = orc.huffman_encode(mtf)
    assert lens[0] > 0 and (osz, esz) == (6, 2)
    assert orc.huffman_decode(lens, osz, esz, pay) == mtf


def test_kat_chains(orc):
    ch = orc.encode_block(b"BANANA")  # :172-260, :367-402
    assert orc.decode_block(ch) == b"BANANA"


# ---- 2. golden vectors ----------------------------------------------------------------------
def test_golden_vectors(orc, golden):
    assert len(golden) >= 50
    for name, g in golden.items():
        ch = orc.encode_block(g["input"])
        assert ch.primary_index == g["pi"], name
        assert ch.bwt == g["bwt"], name
        assert ch.mtf == g["mtf"], name
        assert ch.rle == g["rle"], name
        assert ch.lengths == g["lengths"], name
        assert (ch.orig_size, ch.encoded_size) == (g["orig_size"], g["encoded_size"]), name
        assert ch.payload == g["payload"], name
        assert orc.decode_block(ch) == g["input"], name


def test_golden_config1(golden):
    g = golden["cfg1_tiled_65536"]  # pi 20695, RLE 1061 B, payload 216 B
    assert (g["pi"], len(g["rle"]), g["encoded_size"]) == (20695, 1061, 216)


def test_huffman_tie_rule(orc):
    # 5 equal-frequency symbols -> lengths 2,2,3,3,2 (the list head keeps equal-frequency peers behind it)
    lens, *_ = orc.huffman_encode(b"abcde")
    assert [lens[c] for c in b"abcde"] == [2, 2, 3, 3, 2]


def test_rle_decode_errors(orc):
    assert orc.rle_decode_compute_size(b"") == 0
    assert orc.rle_decode_compute_size(bytes([5, 1, 2])) == 0  # truncated literal
    assert orc.rle_decode_compute_size(bytes([0x80])) == 0  # -128 is a no-op
    assert orc.rle_decode_compute_size(bytes([0xFE])) == 0  # run with no value byte


# ---- 3. live cross-check against the compiled reference -------------------------------------
def _cases(seed, count):
    rng = random.Random(seed)
    for _ in range(count):
        n = rng.choice([1, 2, 3, 5, 31, 127, 128, 129, 131, 257, 1000, 3000])
        kind = rng.randrange(5)
        if kind == 0:
            d = bytes(rng.randrange(256) for _ in range(n))
        elif kind == 1:
            d = bytes(rng.choice(b"ab") for _ in range(n))
        elif kind == 2:
            d = b""
            while len(d) < n:
                d += bytes([rng.randrange(3)]) * rng.choice([1, 2, 3, 128, 129, 130, 131, 256, 259])
            d = d[:n]
        elif kind == 3:
            p = rng.randrange(1, 7)
            u = bytes(rng.randrange(3) for _ in range(p))
            d = (u * (n // p + 1))[:n]
        else:
            d = b"".join(rng.choice([b"et ", b"ut ", b"lorem ", b"ipsum\n"]) for _ in range(n))[:n]
        yield d


@pytest.mark.skipif(not have_ref(), reason="reference build (oracle/_ref) not present")
def test_oracle_vs_reference(orc):
    R = Reference()
    for d in _cases(1234, 300):
        a, b = orc.encode_block(d), R.encode_block(d)
        assert a == b, d[:32]
        assert R.decode_block(b) == d


def _huffman_mutations(orc, seed=7, cases=40):
    """Malformed and edge-case Huffman streams derived from valid ones (truncation, bit flips,
    orig_size off by a few), as (lengths, orig_size, encoded_size, payload) tuples."""
    import random

    rnd = random.Random(seed)
    out = []
    for i in range(cases):
        n = rnd.choice([1, 2, 5, 17, 300, 4000])
        alpha = rnd.choice([2, 3, 16, 200])
        data = bytes(rnd.randrange(alpha) for _ in range(n))
        lens, osz, esz, pay = orc.huffman_encode(data)
        out.append((lens, osz, esz, pay))
        if esz > 1:
            out.append((lens, osz, esz - 1, pay[:-1]))  # truncated
        for _ in range(2):
            if esz:
                b = bytearray(pay)
                k = rnd.randrange(esz)
                b[k] ^= 1 << rnd.randrange(8)
                out.append((lens, osz, esz, bytes(b)))  # bit flip
        out.append((lens, osz + rnd.randrange(1, 4), esz, pay))  # asks for more symbols than coded
        if osz > 1:
            out.append((lens, osz - 1, esz, pay))  # stops one symbol early
        out.append((lens, osz, esz + 2, pay + bytes([rnd.randrange(256), 0])))  # trailing bytes
    return out


@pytest.mark.skipif(not have_ref(), reason="reference build (oracle/_ref) not present")
def test_huffman_decode_malformed_vs_reference(orc):
    ref = Reference()
    for lens, osz, esz, pay in _huffman_mutations(orc):
        assert orc.huffman_decode(lens, osz, esz, pay) == ref.huffman_decode(lens, osz, esz, pay)


# ---- code lengths > 32 bits (bra_huffman.c:227-261, emit :409-425): tests/golden/edge.json ----------
def _edge():
    import json

    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "edge.json")) as f:
        return json.load(f)


def fib_input(nsym: int = 34) -> bytes:
    """The rule of tests/golden/make_edge_golden.py: symbol s repeated F(s + 1) times, ascending."""
    f = [1, 1]
    while len(f) < nsym:
        f.append(f[-1] + f[-2])
    return b"".join(bytes([s]) * f[s] for s in range(nsym))


def test_oracle_huffman_lengths_over_32(orc):
    import hashlib

    g = _edge()["huffman_fib34"]
    data = fib_input()
    assert len(data) == g["size"]
    lens, osz, esz, pay = orc.huffman_encode(data)
    assert max(lens) == g["max_length"] == 33
    assert lens.hex() == g["lengths"] and (osz, esz) == (g["orig_size"], g["encoded_size"])
    assert hashlib.sha256(pay).hexdigest() == g["payload_sha256"]
    # the wrapped canonical codes collide: the reference's decoder cannot rebuild the tree
    assert not g["ref_decodes"]
    assert orc.huffman_decode(lens, osz, esz, pay) is None
