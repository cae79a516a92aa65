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


def frame(payload: bytes, ttl: int = 10, create_time: int = 0, peer_id: bytes | None = None) -> bytes:
    body = msgpack.packb([[_uv(P2P_CONSENSUS), ttl, create_time, list(peer_id) if peer_id is not None else None],
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
