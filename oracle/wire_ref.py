"""wire_ref.py — CPU restatement of the reference's consensus wire format with the `msgpack` package
(1.x, MessagePack spec). TEST INFRASTRUCTURE ONLY: imported by tests/ and bench.py's cpu_baseline
leg as the checker, never by the product path.

Types and field order follow the reference: Subject (src/consensus/types.rs:101-104; View is
{round, height}, :60-63), GossipMessage (src/protocol/mod.rs:44-53, `address` skipped; sign_payload =
signature None, :133-137), RawMessage/Header (src/p2p/protocol.rs:30-70; Consensus header of
p2p/server.rs:187: ttl 10, peer_id None), frame = u32 big-endian size + body (src/p2p/codec.rs:15-53).
The serializer convention (rmp-serde compact: struct = array, Vec<u8>/[u8; N] = array of ints,
Option None = nil, unit variant = [index, []]) is SPEC.md §9's; the reference's own serializer lives
in the unvendored `cryptocurrency-kit`, so the bytes are parity-unpinned against the reference — the
MessagePack encoding itself is pinned by the msgpack package.
"""
from __future__ import annotations

import struct

import msgpack

MESSAGE_TYPES = {"Preprepare": 1, "Prepare": 2, "Commit": 3, "RoundChange": 4}
P2P_CONSENSUS = 4


def _uv(idx: int):
    return [idx, []]


def subject(round_: int, height: int, digest: bytes) -> bytes:
    return msgpack.packb([[round_, height], list(digest)])


def gossip(code: int, create_time: int, msg: bytes, signature: bytes | None, commit_seal: bytes | None) -> bytes:
    return msgpack.packb([_uv(code - 1), create_time, list(msg),
                          list(signature) if signature is not None else None,
                          list(commit_seal) if commit_seal is not None else None])


def frame(payload: bytes, ttl: int = 10, create_time: int = 0, peer_id: bytes | None = None,
          code: int = P2P_CONSENSUS) -> bytes:
    body = msgpack.packb([[_uv(code), ttl, create_time, list(peer_id) if peer_id is not None else None],
                          list(payload)])
    return struct.pack(">I", len(body)) + body


def encode(m: dict) -> tuple[bytes, bytes, bytes]:
    """One Subject-carrying consensus message -> (frame, GossipMessage bytes, sign payload bytes)."""
    s = subject(m["round"], m["height"], m["digest"])
    g = gossip(m["code"], m["create_time"], s, m.get("signature"), m.get("commit_seal"))
    sp = gossip(m["code"], m["create_time"], s, None, m.get("commit_seal"))
    return frame(g, m.get("ttl", 10), m.get("raw_time", 0), m.get("peer_id")), g, sp


def decode(fr: bytes) -> dict | None:
    """frame -> fields, or None when it is not a well-formed Subject-carrying Consensus frame."""
    try:
        if len(fr) < 4 or struct.unpack(">I", fr[:4])[0] != len(fr) - 4:
            return None
        hdr, payload = msgpack.unpackb(fr[4:], strict_map_key=False)
        (uv, ttl, rtime, peer) = hdr
        if uv != [P2P_CONSENSUS, []]:
            return None
        g = msgpack.unpackb(bytes(payload))
        if not 3 <= len(g) <= 5:                 # signature / commit_seal are #[serde(default)]
            return None
        cv, ctime, msg, sig, seal = list(g) + [None] * (5 - len(g))
        if cv[1] != [] or not 1 <= cv[0] <= 3:
            return None
        (rnd, height), digest = msgpack.unpackb(bytes(msg))
        if len(digest) != 32 or (sig is not None and len(sig) != 65) or (seal is not None and len(seal) != 65):
            return None
        return dict(code=cv[0] + 1, create_time=ctime, round=rnd, height=height, digest=bytes(digest),
                    signature=bytes(sig) if sig is not None else None,
                    commit_seal=bytes(seal) if seal is not None else None,
                    ttl=ttl, raw_time=rtime, peer_id=bytes(peer) if peer is not None else None)
    except Exception:
        return None


def split_frames(stream: bytes) -> list[int]:
    """Frame start offsets of a byte stream (MsgPacketCodec::decode's loop), plus the end offset."""
    offs, i = [0], 0
    while i + 4 <= len(stream):
        i += 4 + struct.unpack(">I", stream[i:i + 4])[0]
        offs.append(i)
    return offs


# ---- block-carrying frames (SPEC.md §9b): PrePrepare, Blocks, Sync --------------------------------
P2P_BLOCK, P2P_SYNC = 3, 5


def _addr(a: bytes | None):
    return None if a is None else "0x" + bytes(a).hex()


def tx_obj(t: dict):
    """Transaction, serde field order (types/transaction.rs:16-30)"""
    return [t["nonce"], t["price"], t["gas_limit"], _addr(t.get("recipient")), t["amount"], list(t["payload"]),
            list(t["sig"]) if t.get("sig") is not None else None]


def header_obj(b: dict):
    """Header (types/block.rs:16-36); extra / votes None when absent"""
    return [list(b["prev_hash"]), _addr(b["proposer"]), list(b["root"]), list(b["tx_hash"]), list(b["receipt_hash"]),
            b["bloom"], b["difficulty"], b["height"], b["gas_limit"], b["gas_used"], b["time"],
            list(b["extra"]) if b.get("extra") is not None else None,
            [list(v) for v in b["votes"]] if b.get("votes") is not None else None]


def block_obj(b: dict):
    return [header_obj(b), [tx_obj(t) for t in b["txs"]]]


def preprepare_frame(m: dict):
    """-> (frame, sign payload, GossipMessage bytes) of a Preprepare (preprepare.rs:30-43)"""
    msg = msgpack.packb([[m["round"], m["height"]], block_obj(m["block"])])
    sig = m.get("signature")
    g = msgpack.packb([_uv(0), m["create_time"], list(msg), list(sig) if sig is not None else None, None])
    sp = msgpack.packb([_uv(0), m["create_time"], list(msg), None, None])
    return frame(g, m.get("ttl", 10), m.get("raw_time", 0)), sp, g


def blocks_frame(blocks, ttl: int = 10, raw_time: int = 0) -> bytes:
    return frame(msgpack.packb([block_obj(b) for b in blocks]), ttl, raw_time, code=P2P_BLOCK)


def sync_frame(height: int, ttl: int = 10, raw_time: int = 0) -> bytes:
    return frame(msgpack.packb(height), ttl, raw_time, code=P2P_SYNC)


def _envelope(fr: bytes, code: int):
    if len(fr) < 4 or struct.unpack(">I", fr[:4])[0] != len(fr) - 4:
        return None
    hdr, payload = msgpack.unpackb(fr[4:], strict_map_key=False)
    (uv, ttl, rtime, peer) = hdr
    if uv != [code, []]:
        return None
    return bytes(payload), ttl, rtime


def _bytes(x, n=None):
    b = bytes(x)
    if n is not None and len(b) != n:
        raise ValueError
    return b


def _unaddr(s):
    if not isinstance(s, str) or len(s) != 42 or s[:2] not in ("0x", "0X"):
        raise ValueError
    return bytes.fromhex(s[2:])


def block_from_obj(o):
    hdr, txs = o
    if not 11 <= len(hdr) <= 13:                 # extra / votes #[serde(default)]
        raise ValueError
    hdr = list(hdr) + [None] * (13 - len(hdr))
    b = dict(prev_hash=_bytes(hdr[0], 32), proposer=_unaddr(hdr[1]), root=_bytes(hdr[2], 32),
             tx_hash=_bytes(hdr[3], 32), receipt_hash=_bytes(hdr[4], 32), bloom=hdr[5], difficulty=hdr[6],
             height=hdr[7], gas_limit=hdr[8], gas_used=hdr[9], time=hdr[10],
             extra=_bytes(hdr[11]) if hdr[11] is not None else None,
             votes=[_bytes(v, 65) for v in hdr[12]] if hdr[12] is not None else None, txs=[])
    for t in txs:
        if len(t) != 7:
            raise ValueError
        b["txs"].append(dict(nonce=t[0], price=t[1], gas_limit=t[2],
                             recipient=_unaddr(t[3]) if t[3] is not None else None, amount=t[4],
                             payload=_bytes(t[5]), sig=_bytes(t[6], 65) if t[6] is not None else None))
    return b


def decode_preprepare(fr: bytes) -> dict | None:
    try:
        env = _envelope(fr, P2P_CONSENSUS)
        if env is None:
            return None
        payload, ttl, rtime = env
        g = msgpack.unpackb(payload)
        if not 3 <= len(g) <= 5:
            return None
        cv, ctime, msg, sig, seal = list(g) + [None] * (5 - len(g))
        if cv != [0, []]:
            return None
        (rnd, height), blk = msgpack.unpackb(bytes(msg))
        return dict(round=rnd, height=height, create_time=ctime, ttl=ttl, raw_time=rtime,
                    signature=_bytes(sig, 65) if sig is not None else None, block=block_from_obj(blk))
    except Exception:
        return None


def decode_blocks(fr: bytes):
    try:
        env = _envelope(fr, P2P_BLOCK)
        return None if env is None else [block_from_obj(o) for o in msgpack.unpackb(env[0])]
    except Exception:
        return None


def decode_sync(fr: bytes):
    try:
        env = _envelope(fr, P2P_SYNC)
        if env is None:
            return None
        h = msgpack.unpackb(env[0])
        return h if isinstance(h, int) and h >= 0 else None
    except Exception:
        return None
