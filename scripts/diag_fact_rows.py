#!/usr/bin/env python3
"""Diagnostic (not a test): one layered factored step of NCF(f, L) at B rows vs the
fp32 oracle and a float64 oracle -- for the embedding-table gradients, the rows where
the device and the fp32 oracle disagree beyond the test tolerance, with each row's
batch count and which of the two is closer to float64."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import ncf_oracle as O
    import ncf_amd._lib as L
    from ncf_amd import ops
    from ncf_amd.models import NCF
    f, Lyr, B = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    mt = sys.argv[4] if len(sys.argv) > 4 else "NeuMF-end"
    U, I = 6041, 3707
    seeds = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    for s in range(seeds):
        one(mt, f, Lyr, B, U, I, 19 + s, 3 + s)


def one(mt, f, Lyr, B, U, I, seed, data_seed):
    import ncf_oracle as O
    import ncf_amd._lib as L
    from ncf_amd import ops
    from ncf_amd.models import NCF
    DEV = torch.device("cuda", 0)
    torch.manual_seed(seed)
    ref = O.OracleNCF(U, I, f, Lyr, 0.0, mt)
    torch.manual_seed(seed)
    m = NCF(U, I, f, Lyr, 0.0, mt).to(DEV)
    rng = np.random.default_rng(data_seed)
    users = rng.integers(0, U, B)
    items = np.minimum(rng.zipf(1.3, B) - 1, I - 1)
    labels = (rng.random(B) < 0.2).astype(np.int64)
    _, _, g32 = O.forward_backward(ref, users, items, labels)
    ref64 = ref.double()
    _, _, g64 = O.forward_backward(ref64, users, items, labels)
    flat, lay = ops.ensure_flat(m)
    gflat = torch.zeros(int(lay.total), device=DEV)
    ws = ops.new_workspace(lay, B, DEV)
    ctl = ops.new_ctl(B, DEV)
    rows = ops.pack_rows(torch.as_tensor(users, dtype=torch.int32, device=DEV),
                         torch.as_tensor(items, dtype=torch.int32, device=DEV),
                         torch.as_tensor(labels, dtype=torch.float32, device=DEV))
    st = L.stream_ptr()
    L.check(L.hip().ncf_train_step(L.ctypes.byref(lay), flat.data_ptr(), gflat.data_ptr(), rows.data_ptr(), None,
                                   None, ctl.data_ptr(), B, 1, 0, L.DZ_BCE, ws.data_ptr(), ws.numel() * 4, None, st),
            "train")
    L.check(L.hip().ncf_reduce_slab(L.ctypes.byref(lay), ws.data_ptr(), gflat.data_ptr(), ctl.data_ptr(), st), "reduce")
    torch.cuda.synchronize()
    out = {"fact": bool(ops.fact_mode(lay)), "seed": seed, "tables": {}}
    cnt_u, cnt_i = np.bincount(users, minlength=U), np.bincount(items, minlength=I)
    for (p, off), (name, _) in zip(ops._segments(m, lay), m.named_parameters()):
        if name not in g32:
            continue
        if "embed" not in name:  # tower: device and fp32-oracle error against float64, relative to the tensor's max
            got = gflat[off:off + p.numel()].view_as(p).cpu().numpy().astype(np.float64)
            e64 = g64[name].numpy()
            sc = max(float(np.abs(e64).max()), 1e-30)
            out.setdefault("tower", {})[name] = {"dev_vs_f64_rel": float(np.abs(got - e64).max() / sc),
                                                "f32oracle_vs_f64_rel": float(np.abs(g32[name].numpy() - e64).max() / sc)}
            continue
        got = gflat[off:off + p.numel()].view_as(p).cpu().numpy().astype(np.float64)
        e32 = g32[name].numpy().astype(np.float64)
        e64 = g64[name].numpy()
        scale = np.abs(e64).max()
        bad = np.abs(got - e32) > 1e-6 * scale + 1e-4 * np.abs(e32)
        rows_bad = np.unique(np.nonzero(bad)[0])
        cnt = cnt_i if "item" in name else cnt_u
        info = []
        for r in rows_bad[:12]:
            info.append({"row": int(r), "batch_count": int(cnt[r]), "row_max": float(np.abs(e64[r]).max()),
                         "err_dev_vs_f64": float(np.abs(got[r] - e64[r]).max()),
                         "err_f32oracle_vs_f64": float(np.abs(e32[r] - e64[r]).max())})
        ok = np.ones(len(got), dtype=bool)
        ok[rows_bad] = False
        out["tables"][name] = {"bad_elements": int(bad.sum()), "bad_rows": int(len(rows_bad)), "scale": float(scale),
                               "dev_vs_f64_rel_other_rows": float(np.abs(got[ok] - e64[ok]).max() / scale),
                               "f32oracle_vs_f64_rel_other_rows": float(np.abs(e32[ok] - e64[ok]).max() / scale),
                               "dev_vs_f64_max": float(np.abs(got - e64).max()),
                               "f32oracle_vs_f64_max": float(np.abs(e32 - e64).max()), "rows": info}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
