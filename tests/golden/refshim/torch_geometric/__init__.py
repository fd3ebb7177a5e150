"""Golden-generation stand-in for PyG 2.4.0 (absent from the image); forwards to oracle.pyg_ops."""
