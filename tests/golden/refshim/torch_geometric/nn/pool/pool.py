from oracle.pyg_ops import pool_batch, pool_edge  # noqa: F401
