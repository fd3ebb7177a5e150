"""Write graphs in the DeepRank2 HDF5 layout (``<entry>/<group>/<name>``).

Torch-free, like ``h5extract``, so it runs under any interpreter with h5py.
Used to materialise synthetic datasets (``deeprank2_amd.utils.synthetic``) as
files ``GraphDataset`` reads.

Usage: ``python h5write.py IN.npz OUT.hdf5`` where IN.npz is an
``h5extract`` archive (``__entries__`` = the entry names, one blob of
``"<k>|<group>/<name>"`` arrays, k = entry position).
"""

import sys

import numpy as np


def write(path, graphs, h5py):
    with h5py.File(path, "w") as f5:
        for entry, d in graphs.items():
            g = f5.create_group(entry)
            for name, v in d.items():
                g.create_dataset(name, data=np.asarray(v))


def _main(npz, out):
    import h5py  # noqa: PLC0415
    import h5extract  # noqa: PLC0415  (this script's directory is on sys.path)

    with np.load(npz, allow_pickle=False) as z:
        entries = [str(s) for s in z["__entries__"]]
        graphs = {e: {} for e in entries}
        for key, arr in h5extract.unpack(z).items():
            k, name = key.split("|", 1)
            graphs[entries[int(k)]][name] = arr
    write(out, graphs, h5py)


if __name__ == "__main__":
    if len(sys.argv) != 3:  # noqa: PLR2004
        sys.stderr.write(__doc__)
        sys.exit(2)
    _main(sys.argv[1], sys.argv[2])
