"""TEST INFRASTRUCTURE ONLY -- CPU oracle for the NeuMF training hot path.

Only ``tests/``, ``bench.py``'s ``cpu_baseline`` leg and
``__graft_entry__.smoke()`` may import this module, and only as the checker
(or the timed CPU baseline) -- never as the thing measured or shipped.  The
product (``ncf_amd``) never imports it.

What it restates (reference = YonkaMayonkaZ/NCF, paths relative to its root):

* ``OracleNCF``      -- ``src/ncf/models.py:5-46`` (parameters, init RNG order)
                        and ``:97-118`` (forward), as stock PyTorch CPU ops,
                        which is what the reference runs on a CPU.
* ``bce_mean``       -- ``nn.BCEWithLogitsLoss()`` (``scripts/train_neumf.py:86``).
* ``train_steps``    -- the loop body ``scripts/train_neumf.py:106-118``
                        (zero_grad / fwd / loss / backward / Adam or SGD step).
* ``ng_sample``      -- ``src/data/datasets.py:53-69`` via the C restatement
                        in ``sampler_oracle.c`` (legacy MT19937 + masked
                        rejection); ``ng_sample_py`` is a pure-Python restatement
                        for small cases.
* ``epoch_order``    -- the DataLoader(shuffle=True) protocol
                        (``scripts/train_neumf.py:55``): per epoch one int64
                        ``base_seed`` draw, one int64 sampler seed, then
                        ``randperm`` on a fresh generator; a metrics() pass over
                        the test loader costs one more draw.
* ``metrics_np``     -- ``src/training/metrics.py:4-25`` in numpy.
* ``dropout_masks`` / ``forward_masked`` -- the tower's ``nn.Dropout`` (models.py:23)
                        with the device path's hashed masks (parity of the
                        arithmetic given a mask; the mask bits are not torch's).

Pinning: every function here is checked against the reference's own outputs
(``tests/golden/*.npz``, produced by ``tests/golden/make_golden.py`` importing
the reference in the build container) in ``tests/test_oracle.py``.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch
import torch.nn as nn

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "_build", "libncf_oracle.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", _HERE])
        lib = ctypes.CDLL(path)
        lib.oracle_ng_sample.restype = ctypes.c_int64
        lib.oracle_ng_sample.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                         ctypes.c_int64, ctypes.c_int64, ctypes.c_uint32,
                                         ctypes.c_void_p]
        lib.oracle_mt_words.restype = None
        lib.oracle_mt_words.argtypes = [ctypes.c_uint32, ctypes.c_int64, ctypes.c_void_p]
        _LIB = lib
    return _LIB


# --------------------------------------------------------------------------- model
class OracleNCF(nn.Module):
    """Same parameters, same construction order (hence the same CPU-generator
    draws) and same forward as the reference NCF (models.py:5-46, 97-118)."""

    def __init__(self, user_num, item_num, factor_num, num_layers, dropout, model_type):
        super().__init__()
        self.model_type = model_type
        self.embed_user_GMF = nn.Embedding(user_num, factor_num)
        self.embed_item_GMF = nn.Embedding(item_num, factor_num)
        dm = factor_num * (2 ** (num_layers - 1))
        self.embed_user_MLP = nn.Embedding(user_num, dm)
        self.embed_item_MLP = nn.Embedding(item_num, dm)
        mods = []
        width = factor_num * (2 ** num_layers)
        for _ in range(num_layers):
            mods += [nn.Dropout(p=dropout), nn.Linear(width, width // 2), nn.ReLU()]
            width //= 2
        self.MLP_layers = nn.Sequential(*mods)
        self.predict_layer = nn.Linear(factor_num if model_type in ("GMF", "MLP") else 2 * factor_num, 1)
        for emb in (self.embed_user_GMF, self.embed_item_GMF, self.embed_user_MLP, self.embed_item_MLP):
            nn.init.normal_(emb.weight, std=0.01)
        for m in self.MLP_layers:
            if isinstance(m, nn.Linear):
                nn.init.xavier_uniform_(m.weight)
        nn.init.kaiming_uniform_(self.predict_layer.weight, a=1, nonlinearity="sigmoid")

    def forward(self, user, item):
        if self.model_type == "GMF":
            out = self.embed_user_GMF(user) * self.embed_item_GMF(item)
        elif self.model_type == "MLP":
            out = self.MLP_layers(torch.cat((self.embed_user_MLP(user), self.embed_item_MLP(item)), -1))
        else:
            gmf = self.embed_user_GMF(user) * self.embed_item_GMF(item)
            mlp = self.MLP_layers(torch.cat((self.embed_user_MLP(user), self.embed_item_MLP(item)), -1))
            out = torch.cat((gmf, mlp), -1)
        return self.predict_layer(out).view(-1)


def bce_mean(logits, labels):
    return nn.BCEWithLogitsLoss()(logits, labels.float())


def make_optimizer(model, lr, kind="adam"):
    if kind == "adam":
        return torch.optim.Adam(model.parameters(), lr=lr)
    if kind == "sgd":
        return torch.optim.SGD(model.parameters(), lr=lr)
    raise ValueError(kind)


def train_steps(model, opt, users, items, labels, steps=None):
    """Reference loop body (train_neumf.py:106-118) over pre-formed batches.
    users/items/labels: int64 [T, B] (or lists of 1-D arrays).  Returns losses."""
    losses = []
    T = len(users) if steps is None else steps
    for t in range(T):
        u = torch.as_tensor(np.asarray(users[t]), dtype=torch.int64)
        i = torch.as_tensor(np.asarray(items[t]), dtype=torch.int64)
        y = torch.as_tensor(np.asarray(labels[t]), dtype=torch.int64)
        opt.zero_grad()
        loss = bce_mean(model(u, i), y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    return losses


def forward_backward(model, users, items, labels):
    """One forward + BCE + backward; returns (logits, loss, {name: grad})."""
    model.zero_grad(set_to_none=True)
    u = torch.as_tensor(np.asarray(users), dtype=torch.int64)
    i = torch.as_tensor(np.asarray(items), dtype=torch.int64)
    y = torch.as_tensor(np.asarray(labels), dtype=torch.int64)
    logits = model(u, i)
    loss = bce_mean(logits, y)
    loss.backward()
    grads = {k: p.grad.detach().clone() for k, p in model.named_parameters() if p.grad is not None}
    return logits.detach(), float(loss.item()), grads


# --------------------------------------------------------------------------- dropout
# nn.Dropout(p) before every tower Linear (models.py:23).  torch draws the masks from
# its Philox stream, which nothing here reproduces; the device path hashes them
# (include/ncf_hip.h ncf_dropout_hash) and this restates that hash, so the
# arithmetic given a mask is checked exactly ("parity unpinned" for the mask bits).
_C0, _C1, _C2 = np.uint64(0x9E3779B97F4A7C15), np.uint64(0xBF58476D1CE4E5B9), np.uint64(0x94D049BB133111EB)


def dropout_hash(seed, t, layer, rows, cols):
    """ncf_dropout_hash over rows x cols (uint64 arithmetic wraps like C)."""
    r = np.asarray(rows, dtype=np.int64).astype(np.uint64)[:, None]
    c = np.asarray(cols, dtype=np.uint64)[None, :]
    with np.errstate(over="ignore"):
        x = (np.uint64(seed) << np.uint64(32)) ^ (np.uint64(t) * _C0) ^ (r * _C1) ^ \
            ((np.uint64(layer << 16) | c) * _C2)
        x ^= x >> np.uint64(30)
        x *= _C1
        x ^= x >> np.uint64(27)
        x *= _C2
        x ^= x >> np.uint64(31)
    return (x >> np.uint64(32)).astype(np.uint32)


def dropout_masks(model, seed, t, rows, p):
    """Per tower layer k, the multiplier of each element of its input for the given
    epoch-stream rows at step t: 1 / (1 - p) in fp32 where kept, else 0."""
    p32 = np.float32(p)
    thr = np.uint32(0xFFFFFFFF) if p32 >= 1 else np.uint32(int(float(p32) * 4294967296.0))
    scale = np.float32(0) if p32 >= 1 else np.float32(1) / (np.float32(1) - p32)
    widths = [m.in_features for m in model.MLP_layers if isinstance(m, nn.Linear)]
    return [torch.from_numpy(np.where(dropout_hash(seed, t, k, rows, np.arange(w)) >= thr, scale,
                                      np.float32(0)).astype(np.float32)) for k, w in enumerate(widths)]


def forward_masked(model, user, item, masks):
    """OracleNCF.forward with the tower's Dropout modules replaced by `masks`."""
    def tower(x):
        k = 0
        for m in model.MLP_layers:
            if isinstance(m, nn.Dropout):
                x = x * masks[k]
                k += 1
            else:
                x = m(x)
        return x
    if model.model_type == "GMF":
        out = model.embed_user_GMF(user) * model.embed_item_GMF(item)
    elif model.model_type == "MLP":
        out = tower(torch.cat((model.embed_user_MLP(user), model.embed_item_MLP(item)), -1))
    else:
        gmf = model.embed_user_GMF(user) * model.embed_item_GMF(item)
        out = torch.cat((gmf, tower(torch.cat((model.embed_user_MLP(user), model.embed_item_MLP(item)), -1))), -1)
    return model.predict_layer(out).view(-1)


# --------------------------------------------------------------------------- data stream
def ng_sample(pos_users, pos_items, num_item, num_ng, seed):
    """Negatives of datasets.py:53-69 after np.random.seed(seed) (C restatement)."""
    pu = np.ascontiguousarray(pos_users, dtype=np.int64)
    pi = np.ascontiguousarray(pos_items, dtype=np.int64)
    out = np.empty(len(pu) * num_ng, dtype=np.int64)
    _lib().oracle_ng_sample(pu.ctypes.data, pi.ctypes.data, len(pu), int(num_item), int(num_ng),
                            int(seed) & 0xFFFFFFFF, out.ctypes.data)
    return out


def mt_words(seed, n):
    out = np.empty(n, dtype=np.uint32)
    _lib().oracle_mt_words(int(seed) & 0xFFFFFFFF, int(n), out.ctypes.data)
    return out


def ng_sample_py(pos_users, pos_items, num_item, num_ng, seed):
    """Pure-Python restatement on numpy's own legacy generator (small cases)."""
    rs = np.random.RandomState(seed)
    train = set(zip(np.asarray(pos_users).tolist(), np.asarray(pos_items).tolist()))
    out = []
    for u in np.asarray(pos_users).tolist():
        for _ in range(num_ng):
            j = rs.randint(num_item)
            while (u, j) in train:
                j = rs.randint(num_item)
            out.append(j)
    return np.asarray(out, dtype=np.int64)


def epoch_order(n, gen: torch.Generator | None = None):
    """One DataLoader(shuffle=True) epoch on the global (or given) generator:
    draw base_seed, draw the sampler seed, randperm on a fresh generator."""
    torch.empty((), dtype=torch.int64).random_(generator=gen)           # _BaseDataLoaderIter base_seed
    seed = int(torch.empty((), dtype=torch.int64).random_(generator=gen).item())   # RandomSampler
    g = torch.Generator()
    g.manual_seed(seed)
    return torch.randperm(n, generator=g).numpy()


def test_pass_draw(gen: torch.Generator | None = None):
    """metrics() iterating a non-shuffled DataLoader consumes one base_seed draw."""
    torch.empty((), dtype=torch.int64).random_(generator=gen)


# --------------------------------------------------------------------------- metrics
def metrics_np(logits, items, batch_size, top_k):
    """metrics.py:4-25 on precomputed logits (ties resolved like a stable argsort of
    -logits; fixtures are tie-free).  Returns (HR list[int], NDCG list[float])."""
    logits = np.asarray(logits)
    items = np.asarray(items)
    HR, NDCG = [], []
    for s in range(0, len(items), batch_size):
        p = logits[s:s + batch_size]
        it = items[s:s + batch_size]
        if top_k > len(p):
            raise RuntimeError("selected index k out of range")
        idx = np.argsort(-p, kind="stable")[:top_k]
        rec = it[idx]
        gt = it[0]
        hit = gt in rec
        HR.append(int(hit))
        NDCG.append(1.0 / np.log2(int(np.where(rec == gt)[0][0]) + 2) if hit else 0.0)
    return HR, NDCG


def flat_state(model):
    return {k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}


# ---------------------------------------------------------------------------
# Knowledge distillation (config C5): restatement of src/distillation/*.py as
# stock torch CPU ops.  Pinned by tests/golden/G8_distill.npz (reference run).

class OracleDistill(nn.Module):
    """``strategy`` in {"response", "feature", "attention", "unified"}.

    * task loss      F.binary_cross_entropy_with_logits        (base.py:36-38)
    * kd(s, t)       MSE(sigmoid(s / T), sigmoid(t / T)) * T^2   (base.py:27-34; Feature- and
                     AttentionDistillation inherit it)
    * response       alpha * task + (1 - alpha) * MSE(s, t)      (base.py:40-50; response.py:28-32
                     overrides kd with the plain logit MSE)
    * feature        alpha * task + max(0, 1 - alpha - beta) * kd(s, t) + beta * mean over
                     matched keys of MSE(adapter(student feature), teacher feature)
                     (feature.py:12-147; adapters nn.Linear(S, T) built in key order, :36-46;
                     unmatched keys skipped, :97-106)
    * attention      alpha * task + (1 - alpha - gamma) * kd(s, t) + gamma * mean over keys of
                     KL(softmax_batch(||normalize(f)||) ...)      (attention.py:16-102)
    * unified        the reference file is empty (src/distillation/unified.py, 0 bytes):
                     alpha * task + max(0, 1 - alpha - beta - gamma) * kd + beta * feature
                     + gamma * attention -- this build's definition, parity unpinned.
    """

    def __init__(self, teacher, student, strategy="response", temperature=2.0, alpha=0.5, beta=0.3, gamma=0.2):
        super().__init__()
        self.teacher, self.student = teacher, student
        self.strategy, self.temperature = strategy, temperature
        self.alpha, self.beta, self.gamma = alpha, beta, gamma
        for p in teacher.parameters():
            p.requires_grad = False
        teacher.eval()
        self.adaptation_layers = nn.ModuleDict()
        if strategy in ("feature", "unified"):
            tg, sg = teacher.embed_user_GMF.embedding_dim, student.embed_user_GMF.embedding_dim
            if tg != sg:
                self.adaptation_layers["gmf_features"] = nn.Linear(sg, tg)
            tm = teacher.embed_user_MLP.embedding_dim + teacher.embed_item_MLP.embedding_dim
            sm = student.embed_user_MLP.embedding_dim + student.embed_item_MLP.embedding_dim
            if tm != sm:
                self.adaptation_layers["mlp_input"] = nn.Linear(sm, tm)

    @staticmethod
    def features(model, u, i):
        f = {"gmf_features": model.embed_user_GMF(u) * model.embed_item_GMF(i)}
        x = torch.cat((model.embed_user_MLP(u), model.embed_item_MLP(i)), -1)
        f["mlp_input"] = x
        k = 0
        for layer in model.MLP_layers:
            if isinstance(layer, nn.Linear):
                x = layer(x)
                f[f"mlp_linear_{k}"] = x
                k += 1
            elif isinstance(layer, nn.ReLU):
                x = layer(x)
                f[f"mlp_relu_{k - 1}"] = x
        return f

    def feature_loss(self, tf, sf):
        tot, cnt = 0, 0
        for key, t in tf.items():
            if key not in sf:
                continue
            s = sf[key]
            if t.shape != s.shape:
                if key not in self.adaptation_layers:
                    continue
                s = self.adaptation_layers[key](s)
            tot = tot + torch.nn.functional.mse_loss(s, t)
            cnt += 1
        return tot / cnt if cnt else torch.tensor(0.0)

    @staticmethod
    def attention_loss(tf, sf):
        def att(x):
            a = torch.norm(torch.nn.functional.normalize(x, p=2, dim=-1), p=2, dim=-1, keepdim=True)
            return torch.nn.functional.softmax(a, dim=0)
        tot, cnt = 0, 0
        for key in ("gmf_features", "mlp_input"):
            ta, sa = att(tf[key]).view(-1) + 1e-8, att(sf[key]).view(-1) + 1e-8
            ta, sa = ta / ta.sum(), sa / sa.sum()
            tot = tot + torch.nn.functional.kl_div(torch.log(sa), ta, reduction="batchmean")
            cnt += 1
        return tot / max(cnt, 1)

    def forward(self, u, i, y):
        with torch.no_grad():
            tl = self.teacher(u, i)
            tf = self.features(self.teacher, u, i)
        sl = self.student(u, i)
        task = torch.nn.functional.binary_cross_entropy_with_logits(sl, y)
        a, b, g = self.alpha, self.beta, self.gamma
        if self.strategy == "response":
            return a * task + (1 - a) * torch.nn.functional.mse_loss(sl, tl)
        T = self.temperature
        resp = torch.nn.functional.mse_loss(torch.sigmoid(sl / T), torch.sigmoid(tl / T)) * (T ** 2)
        sf = self.features(self.student, u, i)
        if self.strategy == "feature":
            return a * task + max(0, 1 - a - b) * resp + b * self.feature_loss(tf, sf)
        if self.strategy == "attention":
            return a * task + (1 - a - g) * resp + g * self.attention_loss(tf, sf)
        return (a * task + max(0, 1 - a - b - g) * resp + b * self.feature_loss(tf, sf)
                + g * self.attention_loss(tf, sf))
