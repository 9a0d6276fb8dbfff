"""src.data.datasets (reference src/data/datasets.py) -> ncf_amd.data."""
from ncf_amd.data import NCFData, load_all  # noqa: F401
