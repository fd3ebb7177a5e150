from oracle.pyg_ops import max_pool_x  # noqa: F401
