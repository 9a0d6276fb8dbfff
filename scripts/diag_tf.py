"""Diagnostics: teacher-forced C4 steps, dump the elements that differ."""
import sys, os
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from oracle import ncf_oracle as O
import test_gpu_parity as P
from ncf_amd import ops
C4_U, C4_I = P.C4_U, P.C4_I
T, B = int(sys.argv[1]) if len(sys.argv) > 1 else 4, 16384
ref, m, eng = P._engine_for("NeuMF-end", 16, 3, C4_U, C4_I, 15)
rng = np.random.default_rng(41)
users = rng.integers(0, C4_U, (20, B)); items = np.minimum(rng.zipf(1.2, (20, B)) - 1, C4_I - 1)
labels = (rng.random((20, B)) < 0.2).astype(np.int64)
P._stream(eng, users, items, labels, B)
opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
segs = ops._segments(m, eng.lay)
for t in range(T):
    with torch.no_grad():
        for (p, off), (k, rp) in zip(segs, ref.named_parameters()):
            n = rp.numel()
            eng.flat[off:off + n].copy_(rp.detach().reshape(-1))
            st = opt.state.get(rp, {})
            eng.exp_avg[off:off + n].copy_(st["exp_avg"].reshape(-1) if st else torch.zeros(n))
            eng.exp_avg_sq[off:off + n].copy_(st["exp_avg_sq"].reshape(-1) if st else torch.zeros(n))
    mom = {k: opt.state[rp]["exp_avg"].clone() if rp in opt.state else None for k, rp in ref.named_parameters()}
    pres = []
    hs = [mm.register_forward_hook(lambda mod, i, o: pres.append(o.detach())) for mm in ref.MLP_layers
          if isinstance(mm, torch.nn.Linear)]
    with torch.no_grad():
        ref(torch.as_tensor(users[t]), torch.as_tensor(items[t]))
    for h in hs:
        h.remove()
    mins = torch.stack([p.abs().min(dim=1).values for p in pres]).min(dim=0).values.numpy()
    order = np.argsort(mins)[:8]
    print(f"step {t}: smallest |pre| per sample:", [(int(users[t][r]), int(items[t][r]), f"{mins[r]:.2e}") for r in order])
    eng.ctl[0] = t; eng.ctl[1] = t
    eng.run(1, use_graph=False)
    O.train_steps(ref, opt, [users[t]], [items[t]], [labels[t]])
    torch.cuda.synchronize()
    for (p, off), (k, rp) in zip(segs, ref.named_parameters()):
        got = eng.flat[off:off + p.numel()].cpu().numpy().reshape(rp.shape)
        exp = rp.detach().numpy()
        bad = np.abs(got - exp) > 1e-5 * np.abs(exp) + 5e-6
        if bad.any():
            g = rp.grad.numpy()
            idx = np.argwhere(bad)
            rowsb = np.unique(idx[:, 0]) if idx.shape[1] > 1 else idx
            print(f"step {t} {k}: {bad.sum()} bad, rows {rowsb[:10].tolist()} ({len(rowsb)} rows)")
            for r in rowsb[:4]:
                r = int(r)
                if exp.ndim == 2:
                    cols = np.flatnonzero(bad[r])
                    occ = int((users[t] == r).sum()) if "user" in k else int((items[t] == r).sum())
                    print(f"   row {r}: {len(cols)} cols bad, occurrences in batch {occ}, |g| row max {np.abs(g[r]).max():.3e}")
                    for c in cols[:4]:
                        mm = None if mom[k] is None else float(mom[k][r, c])
                        print(f"      col {c}: got {got[r,c]:.6e} exp {exp[r,c]:.6e} g_ref {g[r,c]:.3e} m_prev {mm}")
print("done")
