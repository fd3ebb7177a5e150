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
datasets), split over worker processes (each opens the file read-only).  A
contiguous dataset (DeepRank2 writes no chunked or compressed ones) is not
read through HDF5 at all: the workers report its file offset, dtype and shape
(``h5d.get_offset``), and the reader takes its bytes from a read-only memory
map of the file (``np.memmap``: only the pages of the extracted datasets are
read and stay resident, not the file's names, metadata and free space);
anything else is read by ``h5d.read``
into the archive's blob.  The reference instead reopens the file and reads
every feature per item (``dataset.py:893-1052``, ~2.5 ms per graph on one
core).

Archive layout (a handful of arrays whatever the number of datasets, so the
archive loads in one read): ``__entries__`` ("<file-index>\t<entry>"),
``__files__`` (paths), ``__names__`` ("<k>|<group>/<name>", k = the entry's
position in ``__entries__``), ``__dtypes__``, ``__shapes__`` (flattened) with
``__ndim__``, ``__src__`` (-1: the bytes are in ``__blob__``; f >= 0: in file
f at the offset), ``__offsets__`` (byte offsets into ``__blob__`` or the
file) and ``__blob__``.  String datasets (``_name``, ``_chain_id``) are
skipped.

Usage: ``python h5extract.py OUT.npz FILE.hdf5 [FILE.hdf5 ...]``
"""

import os
import sys

import numpy as np

GROUPS = ("node_features", "edge_features", "target_values", "clustering")


def _read_entries(args):
    """Worker: (file index, path, [(k, entry)]) -> [(k, "group/name", src)] with
    src = (dtype str, shape, file index, byte offset) for a contiguous dataset,
    else the array (low-level h5py)."""
    import h5py  # noqa: PLC0415

    fi, path, todo = args
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
                shape = dsid.shape
                off = dsid.get_offset()
                nbytes = int(np.prod(shape, dtype=np.int64)) * dt.itemsize
                if off is not None and dsid.get_storage_size() == nbytes and nbytes > 0:
                    out.append((k, name.decode(), (dt.str, tuple(shape), fi, int(off))))
                else:
                    arr = np.empty(shape, dtype=dt)
                    if nbytes:
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


def read_index(paths, workers=None):
    """Every entry of every file: (entries ["<file-index>\t<entry>"], records
    [(k, "group/name", src)] in entry order; src as in _read_entries)."""
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
        jobs += [(fi, str(p), todo[i : i + step]) for i in range(0, len(todo), step)]
    if len(jobs) > 1:
        import multiprocessing as mp  # noqa: PLC0415

        with mp.get_context("fork").Pool(min(len(jobs), 16)) as pool:
            parts = pool.map(_read_entries, jobs)
    else:
        parts = [_read_entries(j) for j in jobs]
    return entries, [r for part in parts for r in part]


def read_arrays(paths, workers=None):
    """As read_index, with every record's array (file-offset records as views
    into one read of their file)."""
    entries, records = read_index(paths, workers)
    bufs = {}
    out = []
    for k, name, src in records:
        if isinstance(src, tuple):
            dt, shape, fi, off = src
            if fi not in bufs:
                bufs[fi] = np.memmap(paths[fi], dtype=np.uint8, mode="r")  # pages read as touched: only the extracted bytes stay resident
            dtype = np.dtype(dt)
            # a private copy: the caller caches these, and a view would see (or
            # SIGBUS on) an HDF5 file rewritten in place while it is alive
            src = np.frombuffer(bufs[fi], dtype=dtype, count=int(np.prod(shape, dtype=np.int64)), offset=off).reshape(shape).copy()
        out.append((k, name, src))
    return entries, out


def pack(entries, records, paths):
    """The archive's arrays (see the module docstring) from (k, name, src) records."""
    n = len(records)
    src = np.full(n, -1, dtype=np.int64)
    offsets = np.zeros(n + 1, dtype=np.int64)
    dts, shapes, ndims = [], [], np.zeros(n, dtype=np.int64)
    pos = 0
    blobs = []
    for i, (_, _, r) in enumerate(records):
        if isinstance(r, tuple):
            dt, shape, fi, off = r
            src[i], offsets[i] = fi, off
        else:
            a = np.asarray(r)
            dt, shape = a.dtype.str, a.shape  # (before ascontiguousarray, which makes 0-d arrays 1-d)
            a = np.ascontiguousarray(a)
            offsets[i] = pos
            blobs.append(a.reshape(-1).view(np.uint8))
            pos += a.nbytes
        dts.append(dt)
        shapes.extend(shape)
        ndims[i] = len(shape)
    offsets[n] = pos
    blob = np.concatenate(blobs) if blobs else np.zeros(0, dtype=np.uint8)
    return {
        "__entries__": np.array(entries, dtype=np.str_),
        "__files__": np.array([str(p) for p in paths], dtype=np.str_),
        "__names__": np.array([f"{k}|{nm}" for k, nm, _ in records], dtype=np.str_),
        "__dtypes__": np.array(dts, dtype=np.str_),
        "__ndim__": ndims,
        "__shapes__": np.array(shapes, dtype=np.int64),
        "__src__": src,
        "__offsets__": offsets,
        "__blob__": blob,
    }


def unpack(z):
    """Inverse of :func:`pack`: {"<k>|<group>/<name>": array} (views into the
    blob, or into one read of each source file)."""
    blob, offsets, ndim, shapes = z["__blob__"], z["__offsets__"], z["__ndim__"], z["__shapes__"]
    src = z["__src__"] if "__src__" in z else np.full(ndim.size, -1, dtype=np.int64)
    files = [str(f) for f in z["__files__"]]
    ends = np.cumsum(ndim)
    bufs = {}
    dtypes = {}
    out = {}
    for i, (name, dt) in enumerate(zip(z["__names__"].tolist(), z["__dtypes__"].tolist())):
        nd = int(ndim[i])
        shape = tuple(shapes[ends[i] - nd : ends[i]].tolist())
        dtype = dtypes.get(dt)
        if dtype is None:
            dtype = dtypes[dt] = np.dtype(dt)
        count = 1
        for v in shape:
            count *= v
        f = int(src[i])
        if f < 0:
            buf = blob
        else:
            buf = bufs.get(f)
            if buf is None:
                buf = bufs[f] = np.memmap(files[f], dtype=np.uint8, mode="r")  # pages read as touched, not the whole file pinned
        a = np.frombuffer(buf, dtype=dtype, count=count, offset=int(offsets[i])).reshape(shape) if count else np.empty(shape, dtype=dtype)
        # file-backed arrays are copied out of the map (writable, and immune to
        # the user's HDF5 file being rewritten while the dataset is alive)
        out[name] = a.copy() if (f >= 0 and count) else a
    return out


def extract(out_path, paths):
    entries, records = read_index(paths)
    np.savez(out_path, **pack(entries, records, paths))


if __name__ == "__main__":
    if len(sys.argv) < 3:  # noqa: PLR2004
        sys.stderr.write(__doc__)
        sys.exit(2)
    extract(sys.argv[1], sys.argv[2:])
