from oracle.pyg_ops import Batch, Data  # noqa: F401
