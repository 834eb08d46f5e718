import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import sidekick_amd as sk
from sidekick_amd.quack import fill_splitmix
from oracle import coracle, quack_oracle as qo
n, t, seed = int(float(sys.argv[1])) if len(sys.argv) > 1 else 100_000_000, 32, 0x5EED0005
ctx = sk.get_context(0)
log = torch.empty(n, dtype=torch.int32, device="cuda:0")
fill_splitmix(ctx, log, seed)
h = log.cpu().numpy().view(np.uint32)
print("fill ok", (h[:1000] == coracle.splitmix_u32(seed, 1000)).all(), flush=True)
sent = sk.PowerSumQuackU32(t); sent.insert_batch(log)
t0 = time.time(); want = coracle.encode_u32(h, t); print("oracle s", time.time() - t0, flush=True)
print("sent ok", sent.power_sums() == want, sent.count(), flush=True)
rng = np.random.default_rng(seed)
drops = np.sort(rng.choice(n, size=32, replace=False))
keep = torch.ones(n, dtype=torch.bool, device="cuda:0")
keep[torch.from_numpy(drops).to("cuda:0")] = False
kept = log[keep].contiguous()
recv = sk.PowerSumQuackU32(t); recv.insert_batch(kept)
kh = kept.cpu().numpy().view(np.uint32)
print("kept len", kh.size, "matches np", (kh == np.delete(h, drops)).all(), flush=True)
diff = sent.clone(); diff.sub_assign(recv)
dq = qo.OracleQuack(t)
for i in drops: dq.insert(int(h[i]))
print("diff ok", diff.power_sums() == dq.power_sums, diff.count(), flush=True)
c = diff.to_coeffs()
print("coeffs ok", list(c) == dq.to_coeffs(), flush=True)
hits = diff.root_test(c, log)
print("hits", len(hits), hits[:5], flush=True)
w, nh = coracle.root_test_u32(list(c), h[:2_000_000])
print("oracle hits in first 2e6", w.tolist(), "gpu", [x for x in hits if x < 2_000_000], flush=True)
small = diff.root_test(c, log[:2_000_000])
print("gpu on 2e6 prefix", small, flush=True)
