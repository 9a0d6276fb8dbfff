"""src.distillation.feature (reference) -> ncf_amd.distill."""
from ncf_amd.distill import FeatureDistillation  # noqa: F401
