"""Consensus wire codec on the CPU: the host build of the codec source the GPU
kernels share (consensus-rs_amd/csrc/bft_wire.h) against the msgpack-based oracle
(oracle/wire_ref.py), the frame splitter, malformed frames, and the library's exported symbols."""
import os
import random
import re
import struct
import sys

import msgpack

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "consensus-rs_amd"))
import wire_ref as R  # noqa: E402
import wire_lib as W  # noqa: E402

EDGE_INTS = [0, 1, 5, 127, 128, 255, 256, 65535, 65536, 2 ** 32 - 1, 2 ** 32, 2 ** 64 - 1]


def random_message(rng, peer=True):
    code = rng.choice([2, 3, 4])
    m = dict(code=code, round=rng.choice(EDGE_INTS), height=rng.choice(EDGE_INTS[1:] + [100, 70000, 2 ** 40]),
             digest=bytes(rng.randrange(256) for _ in range(32)),
             create_time=rng.choice([0, 1536517089000, 2 ** 63, 2 ** 64 - 1]), ttl=rng.choice([10, 0, 300]),
             raw_time=rng.choice([0, 1536517089000]))
    if code == 4:
        m["digest"] = bytes(32)                     # RoundChange carries EMPTY_HASH (round_change.rs:55-58)
    if rng.random() < 0.8:
        m["signature"] = bytes(rng.randrange(256) for _ in range(65))
    if code == 3 and rng.random() < 0.8:
        m["commit_seal"] = bytes(rng.randrange(256) for _ in range(65))
    if peer and rng.random() < 0.2:
        m["peer_id"] = bytes(rng.randrange(256) for _ in range(34))
    return m


def test_host_codec_matches_msgpack_oracle():
    rng = random.Random(3)
    for _ in range(400):
        m = random_message(rng)
        f, g, sp = W.encode(m)
        assert (f, g, sp) == R.encode(m)
        assert W.decode(f) == R.decode(f) == {**{k: m.get(k) for k in ("signature", "commit_seal", "peer_id")},
                                              **{k: m[k] for k in ("code", "create_time", "round", "height",
                                                                   "digest", "ttl", "raw_time")}}


def test_largest_frame_fits_max_msg_size():
    """codec.rs:12 MAX_MSG_SIZE = 1024: the largest Subject frame (all fields at their widest) fits."""
    big = dict(code=3, round=2 ** 64 - 1, height=2 ** 64 - 1, digest=b"\xff" * 32, create_time=2 ** 64 - 1,
               signature=b"\xff" * 65, commit_seal=b"\xff" * 65, raw_time=2 ** 64 - 1, ttl=2 ** 64 - 1)
    f, g, sp = W.encode(big)
    assert f == R.encode(big)[0]
    assert len(f) <= 1028 and len(g) < 512 and len(g) < 4 * 136    # the GPU slots: 1088-byte frames, 4 Keccak blocks


def test_view_field_order_round_then_height():
    """types.rs:60-63 declares View { round, height }: the Subject array starts [[round, height], ...]."""
    s = R.subject(7, 9, bytes(32))
    assert s[:4] == bytes([0x92, 0x92, 7, 9])


def test_malformed_frames_rejected():
    rng = random.Random(5)
    m = random_message(rng, peer=False)
    m["code"] = 3
    f = W.encode(m)[0]
    assert W.decode(f) is not None
    assert W.decode(f[:-1]) is None                                  # truncated
    assert W.decode(struct.pack(">I", len(f) - 3) + f[4:] + b"\x00") is None    # trailing byte
    bad = bytearray(f)
    bad[6:9] = bytes([0x92, 0x03, 0x90])                             # P2PMsgCode::Consensus -> Block
    assert W.decode(bytes(bad)) is None and R.decode(bytes(bad)) is None
    pp = R.frame(R.gossip(1, 0, R.subject(0, 1, bytes(32)), None, None))   # a Preprepare code: out of scope
    assert W.decode(pp) is None and R.decode(pp) is None
    for cut in range(4, len(f), 17):                                 # every truncation is rejected, never crashes
        assert W.decode(struct.pack(">I", cut - 4) + f[4:cut]) is None


def test_short_gossip_arrays_default_to_none():
    # GossipMessage.signature / commit_seal are #[serde(default)] (protocol/mod.rs:48-51): a 3- or
    # 4-element array decodes with None for the missing options; 2 or 6 elements are rejected
    rng = random.Random(6)
    m = random_message(rng, peer=False)
    m["code"] = 3
    sub = R.subject(m["round"], m["height"], m["digest"])
    for k in (3, 4):
        g = msgpack.packb([[m["code"] - 1, []], m["create_time"], list(sub), list(m["signature"])][:k])
        f = R.frame(g, ttl=m["ttl"], create_time=m["raw_time"])
        want, got = R.decode(f), W.decode(f)
        assert want is not None and want["commit_seal"] is None
        assert (want["signature"] is None) == (k == 3)
        assert got is not None and got["digest"] == want["digest"] and got["round"] == want["round"]
        assert got["signature"] == want["signature"] and got["commit_seal"] is None
    for k in (2, 6):
        g = msgpack.packb(([[m["code"] - 1, []], m["create_time"], list(sub), None, None, None])[:k])
        f = R.frame(g, ttl=m["ttl"], create_time=m["raw_time"])
        assert R.decode(f) is None and W.decode(f) is None


def test_split_frames_matches_codec_loop():
    from bftsim import wire
    rng = random.Random(8)
    frames = [W.encode(random_message(rng))[0] for _ in range(50)]
    stream = b"".join(frames)
    offs = wire.split_frames(stream + frames[0][:7])                 # an incomplete tail frame waits
    assert list(offs) == R.split_frames(stream)
    assert len(offs) == 51 and offs[-1] == len(stream)
    assert list(wire.split_frames(stream, max_frames=5)) == R.split_frames(stream)[:6]


def test_libbftwire_exports_every_declared_symbol():
    from bftsim import wire
    src = open(os.path.join(ROOT, "include", "bftwire.h")).read()
    syms = sorted(set(re.findall(r"\b(bftwire_[a-z0-9_]+)\s*\(", src)))
    L = wire.lib()
    assert len(syms) == 12        # Subject codec (6) + Preprepare / Block / Sync encoders and decoders (6)
    assert not [s for s in syms if not hasattr(L, s)]
    assert L.bftwire_create(0, None) < 0
