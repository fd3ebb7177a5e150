"""The inert checkpoint reader (deeprank2_amd/io/checkpoint.py) on tensor
records whose view geometry is malformed: it must refuse them before any
strided view is built (a crafted offset / stride would otherwise read outside
the storage buffer)."""

from __future__ import annotations

import io
import zipfile

import numpy as np
import pytest

from deeprank2_amd.io.checkpoint import CheckpointFormatError, _rebuild_tensor


def _zip(values):
    buf = io.BytesIO()
    with zipfile.ZipFile(buf, "w") as zf:
        zf.writestr("archive/data/0", np.asarray(values, dtype=np.float32).tobytes())
    buf.seek(0)
    return zipfile.ZipFile(buf)


def _rec(offset, size, stride, numel=6):
    return (("FloatStorage", "0", numel), offset, size, stride, False, None)


def test_valid_views():
    zf = _zip(np.arange(6))
    np.testing.assert_array_equal(_rebuild_tensor(zf, "archive/", _rec(0, (2, 3), (3, 1))).numpy(), np.arange(6).reshape(2, 3))
    np.testing.assert_array_equal(_rebuild_tensor(zf, "archive/", _rec(1, (2, 2), (1, 2))).numpy(), [[1, 3], [2, 4]])
    assert float(_rebuild_tensor(zf, "archive/", _rec(5, (), ()))) == 5.0
    assert _rebuild_tensor(zf, "archive/", _rec(6, (0, 3), (3, 1))).shape == (0, 3)
    np.testing.assert_array_equal(_rebuild_tensor(zf, "archive/", _rec(2, (3,), (0,))).numpy(), [2, 2, 2])  # expanded view


@pytest.mark.parametrize(
    ("offset", "size", "stride"),
    [
        (-1, (2,), (1,)),  # negative offset (would wrap around raw[offset:])
        (0, (2, 3), (4, 1)),  # last element 4 + 2 = 6 is past the storage
        (5, (2,), (1,)),  # offset + 1 = 6
        (6, (), ()),  # a scalar past the end
        (0, (3,), (-1,)),  # negative stride
        (0, (-2,), (1,)),  # negative size
        (0, (2, 2), (1,)),  # rank mismatch
        (7, (0,), (1,)),  # empty view starting past the end
        (0, (1 << 40,), (1,)),  # huge size
    ],
)
def test_malformed_views_are_refused(offset, size, stride):
    zf = _zip(np.arange(6))
    with pytest.raises(CheckpointFormatError):
        _rebuild_tensor(zf, "archive/", _rec(offset, size, stride))


def test_storage_size_mismatch_is_refused():
    zf = _zip(np.arange(6))
    with pytest.raises(CheckpointFormatError):
        _rebuild_tensor(zf, "archive/", _rec(0, (6,), (1,), numel=7))
