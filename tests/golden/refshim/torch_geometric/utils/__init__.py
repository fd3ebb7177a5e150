from oracle.pyg_ops import pyg_scatter as scatter  # noqa: F401
