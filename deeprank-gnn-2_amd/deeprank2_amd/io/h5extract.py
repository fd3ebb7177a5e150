"""Dump DeepRank2 graph HDF5 files to a flat ``.npz`` archive.

This module is deliberately free of torch and of the rest of the package, so it
can run under any interpreter that has ``h5py`` (in this image only
``/opt/conda/bin/python3.9`` does).  :mod:`deeprank2_amd.io.hdf5` calls it in a
subprocess and the graph store is then built from the ``.npz`` with numpy only.

Layout read (writer: reference ``deeprank2/utils/graph.py:210-264``; reader:
``deeprank2/dataset.py:893-1042``)::

    <entry>/node_features/<name>       [N] or [N, k]   (``_position`` [N,3])
    <entry>/edge_features/_index       [E/2, 2] int64  (each contact stored once)
    <entry>/edge_features/<name>       [E/2] or [E/2, k]
    <entry>/target_values/<name>       scalar
    <entry>/clustering/<method>/depth_{0,1}

Archive layout: ``__entries__`` (unicode array of "<file-index>\\t<entry>"),
``__files__`` (unicode array of paths), and one array per dataset under the key
``"<k>|<group>/<name>"`` where ``k`` is the entry's position in ``__entries__``.
String datasets (``_name``, ``_chain_id``) are skipped.

Usage: ``python h5extract.py OUT.npz FILE.hdf5 [FILE.hdf5 ...]``
"""

import sys

import numpy as np

GROUPS = ("node_features", "edge_features", "target_values", "clustering")


def _walk(group, prefix, out, k):
    for name in group:
        obj = group[name]
        path = f"{prefix}/{name}" if prefix else name
        if hasattr(obj, "keys"):
            _walk(obj, path, out, k)
            continue
        val = obj[()]
        arr = np.asarray(val)
        if arr.dtype.kind in ("S", "O", "U"):
            continue
        out[f"{k}|{path}"] = arr


def extract(out_path, paths):
    import h5py  # noqa: PLC0415  (only present in some interpreters)

    arrays = {}
    entries = []
    for fi, p in enumerate(paths):
        with h5py.File(p, "r") as f5:
            for entry in f5:
                k = len(entries)
                entries.append(f"{fi}\t{entry}")
                grp = f5[entry]
                for g in GROUPS:
                    if g in grp:
                        _walk(grp[g], g, arrays, k)
    arrays["__entries__"] = np.array(entries, dtype=np.str_)
    arrays["__files__"] = np.array([str(p) for p in paths], dtype=np.str_)
    np.savez(out_path, **arrays)


if __name__ == "__main__":
    if len(sys.argv) < 3:  # noqa: PLR2004
        sys.stderr.write(__doc__)
        sys.exit(2)
    extract(sys.argv[1], sys.argv[2:])
