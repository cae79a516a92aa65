"""The reference's own unit tests on the hot path, restated against libbftsim's host helpers
(include/bftsim.h) and the oracle: quorum (validator.rs:290-317), sort order (validator.rs:169-193),
View ordering (consensus/types.rs:166-353), MessageType order (protocol/mod.rs:241-250)."""
import ctypes

import pytest

import oracle_lib as O
from bftsim import runtime
from bftsim.configs import C_ADDRESSES, cfg1, sorted_addresses, string_to_address


def addr_from_u64(v):   # Address::from(u64): big-endian in the low bytes
    return v.to_bytes(20, "big")


def test_two_thirds_majority_reference_table():
    L = runtime.lib()
    # validator.rs:301-315
    assert L.bftsim_two_thirds_majority(5) == 3
    assert L.bftsim_two_thirds_majority(3) == 2
    assert 4 >= L.bftsim_two_thirds_majority(5) + 1       # has_two_thirds_majority(4), N=5
    assert not 3 >= L.bftsim_two_thirds_majority(5) + 1
    assert not 2 >= L.bftsim_two_thirds_majority(3) + 1
    # SURVEY §8 table and the f32 formula for every N up to 100k
    for n, q in [(4, 2), (5, 3), (7, 4), (64, 42), (256, 170)]:
        assert L.bftsim_two_thirds_majority(n) == q == O.lib().orc_two_thirds_majority(n)
    import numpy as np
    ns = np.arange(1, 100_001, dtype=np.float32)
    f32 = np.floor(ns * np.float32(2.0) / np.float32(3.0)).astype(np.int64)
    assert (f32 == (2 * np.arange(1, 100_001)) // 3).all()


def test_validator_sort_reference():
    # validator.rs:169-193: [100, 10, 21, 31, 3] → [3, 10, 21, 31, 100]
    got = sorted_addresses([addr_from_u64(v) for v in (100, 10, 21, 31, 3)])
    assert got == [addr_from_u64(v) for v in (3, 10, 21, 31, 100)]
    # the c1..c5 genesis set (examples/c1.toml:14): sorted index c4=0, c1=1, c3=2, c2=3, c5=4
    srt = sorted_addresses([string_to_address(a) for a in C_ADDRESSES])
    order = [srt.index(string_to_address(a)) for a in C_ADDRESSES]
    assert order == [1, 3, 2, 0, 4]
    assert cfg1(True).silent == [4]


def test_string_to_address_reference():
    # common/mod.rs:124-127
    a = string_to_address("0x93908f59c6eff007d228398349214acb6b4ac9a4")
    assert "0x" + a.hex() == "0x93908f59c6eff007d228398349214acb6b4ac9a4"
    with pytest.raises(ValueError):
        string_to_address("0x1234")


@pytest.mark.parametrize("a,b,want", [((1, 1), (1, 1), 0), ((2, 1), (1, 1), 1), ((2, 1), (2, 2), -1),
                                      ((1, 9), (2, 0), -1), ((3, 0), (2, 9), 1)])
def test_view_ordering_reference(a, b, want):
    # consensus/types.rs:81-98, 166-353: lexicographic (height, round)
    assert runtime.lib().bftsim_view_cmp(a[0], a[1], b[0], b[1]) == want


def test_message_type_order_reference():
    """protocol/mod.rs:36-41, 241-250: Preprepare=1 < Prepare < Commit < RoundChange. The order is what
    Core::check_message (core.rs:366-399) acts on: in AcceptRequest only the smallest type (Preprepare)
    passes, every larger one is a FutureMessage; RoundChange compares the height only. Checked as
    behaviour, through the kernels' check_message (libbftsim) and the oracle's, on a grid."""
    L = runtime.lib()
    L.bftsim_check_message.argtypes = [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32]
    OL = O.lib()
    OL.orc_check_message.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int]
    OK, UNKNOWN, FUTURE_BLOCK, OLD, FUTURE_MSG = range(5)
    PREPREPARE, PREPARE, COMMIT, ROUND_CHANGE = 1, 2, 3, 4
    ACCEPT, PREPREPARED, PREPARED, COMMITTED = 1, 2, 3, 4
    for code in (PREPREPARE, PREPARE, COMMIT, ROUND_CHANGE):
        for st in (ACCEPT, PREPREPARED, PREPARED, COMMITTED):
            for core_h in (1, 2, 7):
                for vh in (0, 1, 2, 3, 7, 8):
                    got = L.bftsim_check_message(code, vh, core_h, st)
                    assert got == OL.orc_check_message(code, vh, core_h, st), (code, st, core_h, vh)
                    if vh == 0:
                        assert got == UNKNOWN
                    elif vh > core_h:
                        assert got == FUTURE_BLOCK
                    elif vh < core_h:
                        assert got == OLD
                    elif code == ROUND_CHANGE:
                        assert got == OK                   # round change ignores the state
                    elif st == ACCEPT:
                        # MessageType order: only the smallest code passes before a Preprepare
                        assert got == (OK if code < PREPARE else FUTURE_MSG)
                    else:
                        assert got == OK
    # the order itself: the set of codes a fresh (AcceptRequest) Core accepts at its height is the
    # prefix {Preprepare} of Preprepare < Prepare < Commit, plus RoundChange which skips the state test
    accepted = [c for c in (1, 2, 3, 4) if L.bftsim_check_message(c, 5, 5, ACCEPT) == OK]
    assert accepted == [PREPREPARE, ROUND_CHANGE]
    assert L.bftsim_check_message(9, 5, 5, ACCEPT) < 0     # not a MessageType: EINVAL


def test_proposer_seed_byte_orders():
    """randon_seed (validator.rs:39-48) under both readings of U128::from([u8; 16]) (bigint 4.4.1,
    unvendored): libbftsim's helper, the oracle's and Python integers agree."""
    L = runtime.lib()
    for n in (1, 4, 5, 7, 10, 64, 100, 256):
        for seed in range(40):
            h = bytes(((seed * 53 + i * 29 + 7) & 0xff) for i in range(32))
            buf = h[:8] + bytes(8)
            be = int.from_bytes(buf, "big") % n
            le = int.from_bytes(buf, "little") % n
            assert L.bftsim_seed_from_hash_order(h, n, 0) == O.lib().orc_seed_from_hash_order(h, n, 0) == be
            assert L.bftsim_seed_from_hash_order(h, n, 1) == O.lib().orc_seed_from_hash_order(h, n, 1) == le
    # little-endian: a power-of-two N takes the low bits of hash[0] — not identically 0
    assert len({L.bftsim_seed_from_hash_order(bytes([r] * 32), 64, 1) for r in range(256)}) == 64


def test_proposer_seed_helpers_agree():
    L = runtime.lib()
    for n in (4, 5, 7, 10, 64):
        for seed in range(50):
            h = bytes(((seed * 37 + i * 11) & 0xff) for i in range(32))
            s1 = L.bftsim_seed_from_hash(h, n)
            s2 = O.lib().orc_seed_from_hash(h, n)
            be = int.from_bytes(h[:8], "big")
            assert s1 == s2 == ((be << 64) % n)
            assert L.bftsim_calc_proposer(h, n, 3) == (s1 + 3) % n
    # power-of-two N: seed ≡ 0 ⇒ proposer = round mod N
    for n in (4, 64):
        assert all(L.bftsim_seed_from_hash(bytes([r] * 32), n) == 0 for r in range(256))


def test_keccak_and_genesis_helpers_agree_with_oracle():
    L = runtime.lib()
    from bftsim import _abi
    for m in (b"", b"abc", bytes(range(256)) * 3):
        out = (ctypes.c_uint8 * 32)()
        L.bftsim_keccak256(m, len(m), out)
        assert bytes(out) == O.keccak256(m)
    c = cfg1(True)
    cc, keep = _abi.to_cconfig(c)
    g1 = (ctypes.c_uint8 * 32)()
    L.bftsim_genesis_hash(ctypes.byref(cc), g1)
    oc, keep2 = O.to_orc(c)
    g2 = (ctypes.c_uint8 * 32)()
    O.lib().orc_genesis_hash(ctypes.byref(oc), g2)
    assert bytes(g1) == bytes(g2)
