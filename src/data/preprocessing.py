"""src.data.preprocessing (reference src/data/preprocessing.py) -> ncf_amd.preprocessing."""
from ncf_amd.preprocessing import LeaveOneOutPreprocessor  # noqa: F401
