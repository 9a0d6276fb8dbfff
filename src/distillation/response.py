"""src.distillation.response (reference) -> ncf_amd.distill."""
from ncf_amd.distill import ResponseDistillation, SoftTargetDistillation  # noqa: F401
