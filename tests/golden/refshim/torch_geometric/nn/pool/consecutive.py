from oracle.pyg_ops import consecutive_cluster  # noqa: F401
