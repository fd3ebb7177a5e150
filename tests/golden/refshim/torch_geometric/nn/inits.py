from oracle.pyg_ops import uniform  # noqa: F401
