"""src.ncf.nmf_model (reference src/ncf/nmf_model.py) -> ncf_amd.nmf, plus the
run_nmf_experiment that scripts/evaluate_models.py imports."""
from ncf_amd.nmf import NMFEvaluator, NMFRecommender, run_nmf_experiment  # noqa: F401
