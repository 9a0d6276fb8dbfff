"""src.training: metrics() plus the Trainer the reference's north star asks for."""
from ncf_amd.trainer import Trainer  # noqa: F401
