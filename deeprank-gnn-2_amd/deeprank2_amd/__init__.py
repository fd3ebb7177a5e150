"""deeprank2_amd — MI355X-native DeepRank2 GNN hot path.

Mirrors the reference import paths for the hot path:
``deeprank2_amd.neuralnets.gnn.ginet.GINet`` etc.  ``install_as_deeprank2()``
aliases the modules under the ``deeprank2.*`` names for code written against
the reference.
"""

__version__ = "0.1.0"


def install_as_deeprank2():
    """Register this package's modules under ``deeprank2.*`` in ``sys.modules``."""
    import importlib  # noqa: PLC0415
    import sys  # noqa: PLC0415

    names = [
        "neuralnets", "neuralnets.gnn", "neuralnets.gnn.ginet", "neuralnets.gnn.foutnet",
        "neuralnets.gnn.vanilla_gnn", "neuralnets.gnn.sgat", "neuralnets.gnn.ginet_nocluster",
        "utils", "utils.community_pooling", "utils.earlystopping", "dataset", "trainer",
    ]  # fmt: skip
    renamed = {"utils.exporters": "exporters"}  # deeprank2/utils/exporters.py
    sys.modules.setdefault("deeprank2", sys.modules[__name__])
    for n in names:
        try:
            sys.modules[f"deeprank2.{n}"] = importlib.import_module(f"{__name__}.{n}")
        except ModuleNotFoundError:
            pass
    for ref_name, ours in renamed.items():
        sys.modules[f"deeprank2.{ref_name}"] = importlib.import_module(f"{__name__}.{ours}")
