"""src.ncf.models (reference src/ncf/models.py) -> ncf_amd.models."""
from ncf_amd.models import NCF  # noqa: F401
