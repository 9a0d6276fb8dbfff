"""src.utils.config (reference src/utils/config.py) -> ncf_amd.config."""
from ncf_amd.config import Config, config  # noqa: F401
