"""Output exporters with the reference's interface
(``deeprank2/utils/exporters.py``: ``OutputExporter``,
``OutputExporterCollection``, ``HDF5OutputExporter``).

``HDF5OutputExporter`` keeps the reference's table (phase, epoch, entry,
output, target, loss).  The reference writes it with ``DataFrame.to_hdf``
(PyTables); when PyTables is not importable the same table is written as
``output_exporter_<phase>.csv`` next to where the HDF5 file would be.
"""

from __future__ import annotations

import logging
import os

import pandas as pd

_log = logging.getLogger(__name__)


class OutputExporter:
    def __init__(self, directory_path: str | None = None):
        self._directory_path = directory_path or "./output"
        os.makedirs(self._directory_path, exist_ok=True)

    def __enter__(self):
        return self

    def __exit__(self, exception_type, exception, traceback):  # noqa: ANN001
        pass

    def process(self, pass_name, epoch_number, entry_names, output_values, target_values, loss):
        """entry_names, output_values and target_values have the same length."""

    def is_compatible_with(self, output_data_shape, target_data_shape=None):  # noqa: ARG002
        return True


class OutputExporterCollection:
    def __init__(self, *args):
        self._output_exporters = args

    def __enter__(self):
        for e in self._output_exporters:
            e.__enter__()
        return self

    def __exit__(self, exception_type, exception, traceback):  # noqa: ANN001
        for e in self._output_exporters:
            e.__exit__(exception_type, exception, traceback)

    def process(self, pass_name, epoch_number, entry_names, output_values, target_values, loss):
        for e in self._output_exporters:
            e.process(pass_name, epoch_number, entry_names, output_values, target_values, loss)

    def __iter__(self):
        return iter(self._output_exporters)


class MemoryOutputExporter(OutputExporter):
    """Keeps every ``process`` call in ``self.records`` (no files)."""

    def __init__(self):
        self.records = []

    def process(self, pass_name, epoch_number, entry_names, output_values, target_values, loss):
        self.records.append({"phase": pass_name, "epoch": epoch_number, "entry": list(entry_names), "output": list(output_values), "target": list(target_values), "loss": loss})


class HDF5OutputExporter(OutputExporter):
    def __init__(self, directory_path: str):
        self.phase = None
        super().__init__(directory_path)

    def __enter__(self):
        self.df = pd.DataFrame(data={k: [] for k in ("phase", "epoch", "entry", "output", "target", "loss")})
        return self

    def __exit__(self, exception_type, exception, traceback):  # noqa: ANN001
        if self.phase is None:
            return
        phase = "training" if self.phase == "validation" else self.phase
        try:
            import tables  # noqa: F401, PLC0415

            self.df.to_hdf(os.path.join(self._directory_path, "output_exporter.hdf5"), key=phase, mode="a")
        except ImportError:
            path = os.path.join(self._directory_path, f"output_exporter_{phase}.csv")
            self.df.to_csv(path, index=False)
            _log.info(f"PyTables is not installed: exporter table written to {path}")

    def process(self, pass_name, epoch_number, entry_names, output_values, target_values, loss):
        self.phase = pass_name
        n = len(output_values)
        d = {"phase": [pass_name] * n, "epoch": [epoch_number] * n, "entry": entry_names, "output": output_values, "target": target_values, "loss": [loss] * n}
        self.df = pd.concat([self.df, pd.DataFrame(data=d)]).reset_index(drop=True)
