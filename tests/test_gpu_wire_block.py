"""GPU: the block-carrying frames of libbftwire (bftwire_encode/decode_preprepare, _blocks, _sync;
SPEC.md §9b) bit-exact against the msgpack oracle (oracle/wire_ref.py) and the oracle's Keccak, plus
round trips and malformed frames."""
import os
import random
import struct
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import wire_ref as R  # noqa: E402
import oracle_lib as O  # noqa: E402
from test_wire_block_cpu import rand_block, rand_pp  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def codec():
    from bftsim.wire import Codec
    c = Codec(0)
    yield c
    c.close()


def test_preprepare_batch_matches_oracle(codec):
    from bftsim import wire
    rng = random.Random(11)
    ms = [rand_pp(rng) for _ in range(300)]
    stream, off, sd, mh, ok = codec.encode_preprepare(ms)
    assert bool(ok.all())
    st, off = stream.cpu().numpy().tobytes(), off.cpu().numpy()
    sd, mh = sd.cpu().numpy(), mh.cpu().numpy()
    for i, m in enumerate(ms):
        f, sp, g = R.preprepare_frame(m)
        assert st[off[i]:off[i + 1]] == f, i
        assert bytes(sd[i]) == O.keccak256(sp) and bytes(mh[i]) == O.keccak256(g), i
    arr, dok = codec.decode_preprepare(st, off)
    assert dok.all() and wire.array_to_preprepares(arr) == ms


def test_blocks_and_sync_batches(codec):
    from bftsim import wire
    rng = random.Random(12)
    frames = [[rand_block(rng) for _ in range(rng.randrange(4))] for _ in range(120)]
    stream, off, ok = codec.encode_blocks(frames, ttl=[10] * 120, raw_time=list(range(120)))
    assert bool(ok.all())
    st, off = stream.cpu().numpy().tobytes(), off.cpu().numpy()
    for k, bl in enumerate(frames):
        assert st[off[k]:off[k + 1]] == R.blocks_frame(bl, 10, k), k
    arr, cnt, dok = codec.decode_blocks(st, off, max_per_frame=4)
    assert dok.all()
    for k, bl in enumerate(frames):
        assert [wire.rec_to_block(arr[k, j]) for j in range(cnt[k])] == bl
    hs = [0, 1, 127, 128, 2 ** 32, 2 ** 64 - 1] + [rng.randrange(1 << 40) for _ in range(50)]
    stream, off, ok = codec.encode_sync(hs)
    st, off = stream.cpu().numpy().tobytes(), off.cpu().numpy()
    for i, h in enumerate(hs):
        assert st[off[i]:off[i + 1]] == R.sync_frame(h), i
    got, dok = codec.decode_sync(st, off)
    assert dok.all() and [int(x) for x in got] == hs


def test_hostile_block_frames(codec):
    rng = random.Random(13)
    frames = []
    for i in range(64):
        f, _, _ = R.preprepare_frame(rand_pp(rng))
        kind = i % 4
        if kind == 1:
            cut = rng.randrange(5, len(f))
            f = struct.pack(">I", cut - 4) + f[4:cut]
        elif kind == 2:
            f = bytearray(f)
            f[rng.randrange(4, len(f))] ^= 1 << rng.randrange(8)
            f = bytes(f)
        elif kind == 3:
            f = R.sync_frame(rng.randrange(100))           # another P2P code
        frames.append(f)
    st = b"".join(frames)
    off = np.cumsum([0] + [len(f) for f in frames]).astype(np.int64)
    _, ok = codec.decode_preprepare(st, off)
    for i, f in enumerate(frames):
        assert ok[i] == (R.decode_preprepare(f) is not None), (i, i % 4)
    assert ok[0::4].all() and not ok[1::4].any() and not ok[3::4].any()
