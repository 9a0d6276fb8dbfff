"""NMF baseline of the reference's evaluation scripts (CPU, scikit-learn).

Not on the NeuMF training hot path: ``scripts/evaluate_models.py`` and
``experiments/expQ9.py`` compare NeuMF against it.  The reference's
``src/ncf/nmf_model.py`` defines ``NMFRecommender`` and ``NMFEvaluator`` but not the
``run_nmf_experiment`` that ``scripts/evaluate_models.py:13,180`` imports (an
ImportError on the reference itself).  This module provides
all three, so that script runs unchanged; ``run_nmf_experiment`` is the
factor-sweep loop of ``experiments/expQ9.py:29-53`` with the result keys
evaluate_models.py reads (``hr_mean/hr_std/ndcg_mean/ndcg_std/parameters``).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp


class NMFRecommender:
    """reference src/ncf/nmf_model.py:5-61 (sklearn NMF, random init, MU solver)."""

    def __init__(self, n_components=10, random_state=42, max_iter=300):
        self.n_components = n_components
        self.random_state = random_state
        self.max_iter = max_iter
        self.model = None
        self.user_factors = None
        self.item_factors = None
        self.n_parameters = 0

    def fit(self, train_matrix):
        from sklearn.decomposition import NMF
        dense = train_matrix.toarray() if sp.issparse(train_matrix) else np.asarray(train_matrix)
        dense = np.maximum(dense, 0)
        self.n_users, self.n_items = dense.shape
        self.model = NMF(n_components=self.n_components, random_state=self.random_state, max_iter=self.max_iter,
                         init="random", solver="mu", beta_loss="frobenius")
        self.user_factors = self.model.fit_transform(dense)
        self.item_factors = self.model.components_.T
        self.n_parameters = self.n_users * self.n_components + self.n_items * self.n_components
        print(f"  NMF reconstruction error: {self.model.reconstruction_err_:.4f}")
        return self

    def predict(self, user_ids, item_ids):
        """Dot products of the factor rows; 0.0 for ids outside the fitted matrix
        (nmf_model.py:46-58), vectorised."""
        u = np.asarray(user_ids, dtype=np.int64)
        i = np.asarray(item_ids, dtype=np.int64)
        ok = (u >= 0) & (u < self.n_users) & (i >= 0) & (i < self.n_items)
        out = np.zeros(len(u), dtype=np.float64)
        if ok.any():
            out[ok] = np.einsum("ij,ij->i", self.user_factors[u[ok]], self.item_factors[i[ok]])
        return out

    def get_n_parameters(self):
        return self.n_parameters


class NMFEvaluator:
    """reference src/ncf/nmf_model.py:63-112: candidates grouped by user in first-seen
    order (first item = the positive), ranked by score descending with ties in
    candidate order (Python's stable sort), HR@K / NDCG@K = 1/log2(pos+2)."""

    def __init__(self, model, test_data, train_matrix, top_k=10):
        self.model = model
        self.test_data = test_data
        self.train_matrix = train_matrix
        self.top_k = top_k

    def evaluate(self):
        user_data = {}
        for user, item in self.test_data:
            user_data.setdefault(user, []).append(item)
        hits, ndcgs = [], []
        for user_id, items in user_data.items():
            if user_id >= self.train_matrix.shape[0]:
                continue
            items = np.asarray(items)
            pred = self.model.predict(np.full(len(items), user_id), items)
            ranked = items[np.argsort(-pred, kind="stable")]
            pos = int(np.nonzero(ranked == items[0])[0][0])
            if pos < self.top_k:
                hits.append(1)
                ndcgs.append(1.0 / np.log2(pos + 2))
            else:
                hits.append(0)
                ndcgs.append(0)
        print(f"    Evaluated {len(user_data)} users")
        hr = np.mean(hits) if hits else 0.0
        ndcg = np.mean(ndcgs) if ndcgs else 0.0
        return hr, ndcg


def run_nmf_experiment(train_mat, test_data, n_components_list, num_runs=10, max_iter=500, top_k=10):
    """Factor sweep of experiments/expQ9.py:29-53: for each factor count, num_runs
    fits with random_state 42 + run; mean / std of HR@K and NDCG@K over the runs,
    plus the parameter count (U + I) * factors read by evaluate_models.py:191."""
    results = {}
    for n in n_components_list:
        print(f"Testing {n} factors...")
        hrs, ndcgs = [], []
        params = 0
        for run in range(num_runs):
            nmf = NMFRecommender(n_components=n, random_state=42 + run, max_iter=max_iter)
            nmf.fit(train_mat)
            hr, nd = NMFEvaluator(nmf, test_data, train_mat, top_k).evaluate()
            hrs.append(hr)
            ndcgs.append(nd)
            params = nmf.get_n_parameters()
        results[n] = {"ndcg_mean": float(np.mean(ndcgs)), "ndcg_std": float(np.std(ndcgs)),
                      "hr_mean": float(np.mean(hrs)), "hr_std": float(np.std(hrs)),
                      "parameters": int(params), "max_iterations": int(max_iter)}
        print(f"  {n} factors: HR@10 = {np.mean(hrs):.4f} +/- {np.std(hrs):.4f}, "
              f"NDCG@10 = {np.mean(ndcgs):.4f} +/- {np.std(ndcgs):.4f}")
    return results
