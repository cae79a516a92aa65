"""The reference's per-message path end to end on the GPU, composing the two SURVEY §8f rows:
sender  — Subject / GossipMessage encode (bftwire) -> sign_digest -> Hash::sign (bftsig) -> framed with
          the signature (and, for Commits, the commit seal = sign(block digest), votes.rs:94-101);
receiver — MsgPacketCodec::decode + from_bytes (bftwire) -> sign payload re-encoded from the decoded
          fields -> recover_bytes + public_to_address (bftsig) -> the validator's address
          (GossipMessage::address, protocol/mod.rs:103-116) and verify_address of the seal (commit.rs:96-100).
Keys: the five reference secrets of examples/c1..c5.toml plus seeded ones, so recovered senders are the
genesis validator addresses."""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "consensus-rs_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import wire_ref as R  # noqa: E402
import secp256k1_ref as S  # noqa: E402
import oracle_lib as O  # noqa: E402

pytestmark = pytest.mark.gpu
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "sig_vectors.json")))


def test_message_path_round_trip():
    import torch
    from bftsim.sig import Signer
    from bftsim.wire import Codec
    dev = torch.device("cuda", 0)
    sg, cd = Signer(0), Codec(0)
    n_val, n = 64, 64 * 512                          # 512 views of a 64-validator cluster's votes
    rng = np.random.default_rng(4)
    secs = np.concatenate([np.frombuffer(bytes.fromhex(k["secret"]), np.uint8)[None] for k in GOLD["reference_keys"]]
                          + [rng.integers(0, 128, (n_val - 5, 32), dtype=np.uint8)])
    secs_d = torch.from_numpy(secs).to(dev)
    _, vaddr, vok = sg.secret_to_address(secs_d)
    assert bool((vok == 1).all())
    assert [bytes(a).hex() for a in vaddr[:5].cpu().numpy()] == [k["address"] for k in GOLD["reference_keys"]]
    sender = torch.arange(n, dtype=torch.int32, device=dev) % n_val
    code = torch.from_numpy(rng.choice(np.array([2, 3, 4], dtype=np.uint8), n)).to(dev)
    batch = {"code": code, "round": torch.from_numpy(rng.integers(0, 3, n)).to(dev),
             "height": torch.from_numpy(rng.integers(1, 1000, n)).to(dev),
             "digest": torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).to(dev),
             "create_time": torch.from_numpy(1536517089000 + rng.integers(0, 1 << 20, n)).to(dev)}
    # sender: seal (Commits), sign digest, signature, final frames
    seal, ok = sg.sign(secs_d, batch["digest"], key_index=sender)
    assert bool((ok == 1).all())
    batch["commit_seal"] = seal
    _, _, sd, mh, ok = cd.encode(batch)
    assert bool((ok == 1).all())
    sig, ok = sg.sign(secs_d, sd, key_index=sender)
    assert bool((ok == 1).all())
    frames, offs, _, _, ok = cd.encode({**batch, "signature": sig}, hashes=False)
    assert bool((ok == 1).all())
    # receiver: split (host), decode, re-encode the sign payload, recover, verify the seal
    total = int(offs[-1])
    host = frames[:total].cpu().numpy()
    from bftsim import wire
    assert np.array_equal(wire.split_frames(host, max_frames=n).astype(np.int64), offs.cpu().numpy())
    dec, ok = cd.decode(frames[:total], offs)
    assert bool((ok == 1).all()) and bool((dec["has_sig"] == 1).all())
    rx = {k: dec[k] for k in ("code", "round", "height", "digest", "create_time", "commit_seal")}
    _, _, sd_rx, mh_rx, ok = cd.encode(rx)
    assert torch.equal(sd_rx, sd)                    # the receiver's sign payload is the sender's
    _, addr, ok = sg.recover(sd_rx, dec["signature"], want_pub=False)
    assert bool((ok == 1).all())
    assert torch.equal(addr, vaddr[sender.long()])
    commits = dec["code"] == 3
    seal_ok = sg.verify_address(vaddr[sender.long()][commits], dec["digest"][commits], dec["commit_seal"][commits])
    assert bool((seal_ok == 1).all())
    # a tampered frame (round + 1) still decodes but recovers someone else
    tampered = {**rx, "round": rx["round"] + 1}
    _, _, sd_t, _, _ = cd.encode(tampered)
    _, addr_t, ok_t = sg.recover(sd_t, dec["signature"], want_pub=False)
    assert not bool((addr_t == vaddr[sender.long()]).all(dim=1).any())
    # spot checks against the CPU oracles
    for i in (0, 1, 2, n - 1):
        m = dict(code=int(dec["code"][i]), round=int(dec["round"][i]), height=int(dec["height"][i]),
                 digest=bytes(dec["digest"][i].cpu().numpy()), create_time=int(dec["create_time"][i]),
                 signature=bytes(dec["signature"][i].cpu().numpy()),
                 commit_seal=bytes(dec["commit_seal"][i].cpu().numpy()) if int(dec["code"][i]) == 3 else None,
                 raw_time=int(dec["create_time"][i]))
        f, g, sp = R.encode(m)
        assert bytes(host[int(offs[i]):int(offs[i + 1])]) == f
        assert O.keccak256(sp) == bytes(sd[i].cpu().numpy())
        sec = bytes(secs[i % n_val])
        assert S.sign(sec, O.keccak256(sp)) == bytes(sig[i].cpu().numpy())
    sg.close()
    cd.close()
