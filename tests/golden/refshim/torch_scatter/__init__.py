"""Golden-generation stand-in for torch_scatter 2.1.2; forwards to oracle.pyg_ops."""
from oracle.pyg_ops import scatter_max, scatter_mean, scatter_sum  # noqa: F401
