"""src.distillation.unified: empty in the reference; this build defines it in ncf_amd.distill."""
from ncf_amd.distill import UnifiedDistillation  # noqa: F401
