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

Reading goes through h5py's low-level API (``h5o.visit`` for an entry's
datasets, ``h5d.read`` into preallocated arrays): ~80 us per dataset here
against ~250 us through ``Group.__getitem__`` / ``Dataset.__getitem__``, and
the entries are split over worker processes (each opens the file read-only).
The reference instead reopens the file and reads every feature per item
(``dataset.py:893-1052``, ~2.5 ms per graph on one core).

Archive layout (a handful of arrays whatever the number of datasets, so the
archive loads in one read): ``__entries__`` ("<file-index>\\t<entry>"),
``__files__`` (paths), ``__names__`` ("<k>|<group>/<name>", k = the entry's
position in ``__entries__``), ``__dtypes__``, ``__shapes__`` (flattened) with
``__ndim__``, ``__offsets__`` (byte offsets into ``__blob__``, one more than
datasets) and ``__blob__`` (every dataset's bytes, C order).  String datasets
(``_name``, ``_chain_id``) are skipped.

Usage: ``python h5extract.py OUT.npz FILE.hdf5 [FILE.hdf5 ...]``
"""

import os
import sys

import numpy as np

GROUPS = ("node_features", "edge_features", "target_values", "clustering")


def _read_entries(args):
    """Worker: (path, [(k, entry)]) -> [(k, "group/name", array)] (low-level h5py)."""
    import h5py  # noqa: PLC0415

    path, todo = args
    out = []
    fid = h5py.h5f.open(os.fsencode(path), h5py.h5f.ACC_RDONLY)
    try:
        for k, entry in todo:
            gid = h5py.h5g.open(fid, entry.encode())
            names = []

            def cb(name, info, names=names):
                if info.type == h5py.h5o.TYPE_DATASET and name.split(b"/", 1)[0].decode() in GROUPS:
                    names.append(name)

            h5py.h5o.visit(gid, cb, info=True)
            for name in names:
                dsid = h5py.h5d.open(gid, name)
                dt = dsid.dtype
                if dt.kind in ("S", "O", "U", "V"):
                    continue
                arr = np.empty(dsid.shape, dtype=dt)
                dsid.read(h5py.h5s.ALL, h5py.h5s.ALL, arr)
                out.append((k, name.decode(), arr))
    finally:
        fid.close()
    return out


def _workers(n_entries):
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        cores = min(cores, int(env))
    return max(1, min(cores, 16, n_entries // 64))


def read_arrays(paths, workers=None):
    """Every entry of every file: (entries ["<file-index>\\t<entry>"], records
    [(k, "group/name", array)] in entry order)."""
    import h5py  # noqa: PLC0415

    entries, jobs = [], []
    for fi, p in enumerate(paths):
        with h5py.File(p, "r") as f5:
            names = list(f5.keys())
        todo = []
        for entry in names:
            todo.append((len(entries), entry))
            entries.append(f"{fi}\t{entry}")
        n = workers or _workers(len(todo))
        step = -(-len(todo) // n) if todo else 1
        jobs += [(str(p), todo[i : i + step]) for i in range(0, len(todo), step)]
    if len(jobs) > 1:
        import multiprocessing as mp  # noqa: PLC0415

        with mp.get_context("fork").Pool(min(len(jobs), 16)) as pool:
            parts = pool.map(_read_entries, jobs)
    else:
        parts = [_read_entries(j) for j in jobs]
    return entries, [r for part in parts for r in part]


def pack(entries, records, paths):
    """The archive's arrays (see the module docstring) from (k, name, array) records."""
    sizes = [a.nbytes for _, _, a in records]
    offsets = np.zeros(len(records) + 1, dtype=np.int64)
    offsets[1:] = np.cumsum(sizes)
    blob = np.empty(int(offsets[-1]), dtype=np.uint8)
    for (_, _, a), o in zip(records, offsets[:-1]):
        blob[o : o + a.nbytes] = np.ascontiguousarray(a).reshape(-1).view(np.uint8)
    return {
        "__entries__": np.array(entries, dtype=np.str_),
        "__files__": np.array([str(p) for p in paths], dtype=np.str_),
        "__names__": np.array([f"{k}|{n}" for k, n, _ in records], dtype=np.str_),
        "__dtypes__": np.array([a.dtype.str for _, _, a in records], dtype=np.str_),
        "__ndim__": np.array([a.ndim for _, _, a in records], dtype=np.int64),
        "__shapes__": np.array([s for _, _, a in records for s in a.shape], dtype=np.int64),
        "__offsets__": offsets,
        "__blob__": blob,
    }


def unpack(z):
    """Inverse of :func:`pack`: {"<k>|<group>/<name>": array} (views into the blob)."""
    blob, offsets, ndim, shapes = z["__blob__"], z["__offsets__"], z["__ndim__"], z["__shapes__"]
    out, s = {}, 0
    for i, (name, dt) in enumerate(zip(z["__names__"], z["__dtypes__"])):
        nd = int(ndim[i])
        shape = tuple(int(v) for v in shapes[s : s + nd])
        s += nd
        dtype = np.dtype(str(dt))
        count = int(np.prod(shape, dtype=np.int64)) if nd else 1
        out[str(name)] = np.frombuffer(blob, dtype=dtype, count=count, offset=int(offsets[i])).reshape(shape) if count else np.empty(shape, dtype=dtype)
    return out


def extract(out_path, paths):
    entries, records = read_arrays(paths)
    np.savez(out_path, **pack(entries, records, paths))


if __name__ == "__main__":
    if len(sys.argv) < 3:  # noqa: PLR2004
        sys.stderr.write(__doc__)
        sys.exit(2)
    extract(sys.argv[1], sys.argv[2:])
