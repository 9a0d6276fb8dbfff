"""src.distillation.attention (reference) -> ncf_amd.distill."""
from ncf_amd.distill import AttentionDistillation  # noqa: F401
