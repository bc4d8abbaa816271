import os, sys, ctypes, time
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "indy-plenum_amd"))
from plenum_amd import EdVerifyEngine, pack_messages, synth
oracle = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libed25519_oracle.so"))
eng = EdVerifyEngine(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
pks, sks = eng.seed_keypair_batch(synth.signer_seeds(1000))
msgs, kidx, _ = synth.nym_messages(n, pks, alias_len=43)
buf, off = pack_messages(msgs)
dev = torch.device("cuda", 0)
d_msgs = torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).to(dev)
d_off = torch.from_numpy(off.view(np.int64)).to(dev)
d_sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
d_sk = torch.from_numpy(sks).to(dev); d_k = torch.from_numpy(kidx.astype(np.int32)).to(dev)
eng.sign_batch_device(d_sk, d_k, d_msgs, d_off, n, d_sig)
d_pk = torch.from_numpy(pks).to(dev)[torch.from_numpy(kidx.astype(np.int64)).to(dev)].contiguous()
torch.cuda.synchronize()
sig = d_sig.cpu().numpy()
words = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
eng.verify_batch_device(d_sig, d_pk, d_msgs, d_off, n, words)
torch.cuda.synchronize()
bits = np.unpackbits(words.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool)
bad = np.nonzero(~bits)[0]
print("n", n, "rejected", len(bad), "first", bad[:10], "last", bad[-10:])
for i in list(bad[:3]) + list(bad[-3:]):
    m = msgs[i]
    print(i, "oracle", oracle.oracle_verify_detached(sig[i].tobytes(), m, ctypes.c_uint64(len(m)), pks[kidx[i]].tobytes()))
# host API on the tail
lo = max(0, n - 300)
got = eng.verify_batch(sig[lo:], pks[kidx[lo:]], buf, off[lo:])
print("host-api tail accepted", got.sum(), "/", len(got))
