"""Reference import surface (``from src.ncf.models import NCF`` ...) backed by ncf_amd.

The reference's scripts import ``src.*`` with the repository root on sys.path
(scripts/train_neumf.py:19-24).  These modules re-export the MI355X
implementation under the same names so those scripts run unchanged.
"""
