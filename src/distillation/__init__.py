"""src.distillation (reference src/distillation/__init__.py) -> ncf_amd.distill.
UnifiedDistillation is exported too: scripts/train_student.py imports it, while the
reference's unified.py is empty (see ncf_amd/distill.py)."""
from ncf_amd.distill import (  # noqa: F401
    AttentionDistillation,
    BaseDistillation,
    FeatureDistillation,
    ResponseDistillation,
    SoftTargetDistillation,
    UnifiedDistillation,
)

__all__ = ["BaseDistillation", "ResponseDistillation", "SoftTargetDistillation", "FeatureDistillation",
           "AttentionDistillation", "UnifiedDistillation"]
