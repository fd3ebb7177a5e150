"""HDF5 access for GraphDataset without requiring h5py next to torch.

DeepRank2 graph files (writer ``deeprank2/utils/graph.py:210-264``) are read
once per file into ``{entry: {"group/name": ndarray}}`` (see ``h5extract``).
If ``h5py`` imports in this interpreter it is used directly; otherwise the
extractor runs under an interpreter that has it (``DR_H5PY_PYTHON``, else the
first of ``/opt/conda/bin/python3*`` that imports h5py) and hands back a
``.npz``, read with ``allow_pickle=False``.  Results are cached per
(path, size, mtime) for the life of the process.
"""

from __future__ import annotations

import glob
import os
import subprocess
import sys
import tempfile

import numpy as np

from deeprank2_amd.io import h5extract

_CACHE: dict = {}
_PYTHON = None


def _inprocess_h5py():
    try:
        import h5py  # noqa: PLC0415
    except ImportError:
        return None
    return h5py


def external_python() -> str:
    """An interpreter that can import h5py (raises if none is found)."""
    global _PYTHON  # noqa: PLW0603
    if _PYTHON is not None:
        return _PYTHON
    cands = [os.environ["DR_H5PY_PYTHON"]] if os.environ.get("DR_H5PY_PYTHON") else []
    cands += sorted(glob.glob("/opt/conda/bin/python3*"))
    for c in cands:
        try:
            r = subprocess.run([c, "-c", "import h5py"], capture_output=True, timeout=120, check=False)
        except (OSError, subprocess.TimeoutExpired):
            continue
        if r.returncode == 0:
            _PYTHON = c
            return c
    msg = "reading DeepRank2 HDF5 files needs h5py: none in this interpreter and no DR_H5PY_PYTHON / /opt/conda/bin/python3* with h5py"
    raise RuntimeError(msg)


def _key(path):
    st = os.stat(path)
    return (os.path.abspath(path), st.st_size, st.st_mtime_ns)


def _split_dump(z, n_files):
    """npz written by h5extract -> list (per file) of {entry: {name: array}}."""
    files = [dict() for _ in range(n_files)]
    order = []
    for s in z["__entries__"]:
        fi, entry = str(s).split("\t", 1)
        files[int(fi)][entry] = {}
        order.append((int(fi), entry))
    for key, arr in h5extract.unpack(z).items():
        k, name = key.split("|", 1)
        fi, entry = order[int(k)]
        files[fi][entry][name] = arr
    return files


def read_files(paths) -> list:
    """Per path: {entry: {"group/name": ndarray}} in file order, or an
    ``Exception`` instance if the file could not be read."""
    paths = [str(p) for p in paths]
    out = [None] * len(paths)
    todo = []
    for i, p in enumerate(paths):
        try:
            k = _key(p)
        except OSError as e:
            out[i] = e
            continue
        if k in _CACHE:
            out[i] = _CACHE[k]
        else:
            todo.append(i)
    if not todo:
        return out
    h5py = _inprocess_h5py()
    for i in todo:
        p = paths[i]
        try:
            if h5py is not None:
                ents, recs = h5extract.read_arrays([p], workers=1)  # no fork of this (torch / HIP) process
                entries = {e.split("\t", 1)[1]: {} for e in ents}
                names = [e.split("\t", 1)[1] for e in ents]
                for k, name, arr in recs:
                    entries[names[k]][name] = arr
                res = entries
            else:
                with tempfile.TemporaryDirectory() as td:
                    npz = os.path.join(td, "dump.npz")
                    cmd = [external_python(), h5extract.__file__, npz, p]
                    r = subprocess.run(cmd, capture_output=True, text=True, timeout=3600, check=False)
                    if r.returncode != 0:
                        raise OSError(f"could not read {p}: {r.stderr.strip().splitlines()[-1] if r.stderr.strip() else r.returncode}")  # noqa: TRY301
                    with np.load(npz, allow_pickle=False) as z:
                        res = _split_dump(z, 1)[0]
        except Exception as e:  # noqa: BLE001
            out[i] = e
            continue
        _CACHE[_key(p)] = res
        out[i] = res
    return out


def write_graphs(path, graphs) -> None:
    """Write graphs in the DeepRank2 layout.  ``graphs``: {entry: {"group/name": array}}.
    Uses h5py in-process if present, else the external interpreter."""
    h5py = _inprocess_h5py()
    if h5py is not None:
        from deeprank2_amd.io import h5write  # noqa: PLC0415

        h5write.write(path, graphs, h5py)
        return
    with tempfile.TemporaryDirectory() as td:
        npz = os.path.join(td, "graphs.npz")
        recs = [(k, name, np.asarray(v)) for k, d in enumerate(graphs.values()) for name, v in d.items()]
        np.savez(npz, **h5extract.pack(list(graphs), recs, [str(path)]))
        from deeprank2_amd.io import h5write  # noqa: PLC0415

        r = subprocess.run([external_python(), h5write.__file__, npz, str(path)], capture_output=True, text=True, timeout=3600, check=False)
        if r.returncode != 0:
            msg = f"writing {path} failed: {r.stderr}"
            raise OSError(msg)


if __name__ == "__main__":  # pragma: no cover
    print(read_files(sys.argv[1:]))
