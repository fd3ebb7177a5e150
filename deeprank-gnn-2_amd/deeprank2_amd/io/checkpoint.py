"""Reading DeepRank2 checkpoints without executing anything from the file.

A reference checkpoint (``Trainer._save_model``, deeprank2/trainer.py:926-956,
``torch.save`` zip format) pickles live objects beside the tensors: the
``data_type`` class, the optimizer and loss-function instances
(``state["optimizer"]``, ``state["lossfunction"]``).  ``torch.load(...,
weights_only=True)`` refuses such a file, and a full unpickle would run
whatever callables the file names.  This module reads it another way:
``pickletools.genops`` disassembles ``data.pkl`` and a small stack machine
builds only inert data from the opcodes --

* str / bytes / int / float / bool / None, tuples, lists, dicts, sets;
* tensors from ``torch._utils._rebuild_tensor_v2`` records: the raw storage
  ``data/<key>`` is read from the zip and viewed with numpy (no torch
  deserialisation code runs);
* every other global the file names becomes a :class:`GlobalRef` (module and
  name strings, never imported), and a call of it (``REDUCE`` / ``NEWOBJ``)
  an :class:`Obj` holding the reference and its (inert) arguments and state.

``load_checkpoint`` first tries ``torch.load(weights_only=True)`` (the
checkpoints this package writes load that way) and falls back to the reader.
"""

from __future__ import annotations

import pickletools
import zipfile
from dataclasses import dataclass, field

import numpy as np
import torch

_STORAGE_DTYPES = {
    "FloatStorage": np.float32,
    "DoubleStorage": np.float64,
    "HalfStorage": np.float16,
    "LongStorage": np.int64,
    "IntStorage": np.int32,
    "ShortStorage": np.int16,
    "CharStorage": np.int8,
    "ByteStorage": np.uint8,
    "BoolStorage": np.bool_,
}


@dataclass(frozen=True)
class GlobalRef:
    """A global the pickle names (never imported)."""

    module: str
    name: str

    def __str__(self):
        return f"{self.module}.{self.name}"


@dataclass(eq=False)  # identity hash: an object may key a dict (e.g. an optimizer's param groups)
class Obj:
    """An object the pickle would have constructed: its class and inert arguments / state."""

    cls: GlobalRef
    args: tuple = ()
    state: object = None
    items: dict = field(default_factory=dict)


class _Mark:
    pass


class _NdArray:
    """numpy.ndarray under reconstruction (its BUILD state carries the data)."""

    value = None


_NP_CODES = {"b1", "i1", "u1", "i2", "u2", "i4", "u4", "i8", "u8", "f2", "f4", "f8"}


_MARK = _Mark()


class CheckpointFormatError(ValueError):
    pass


def _rebuild_tensor(zf, prefix, args):
    """torch._utils._rebuild_tensor_v2(storage, offset, size, stride, requires_grad, hooks[, metadata])."""
    storage, offset, size, stride = args[0], int(args[1]), tuple(args[2]), tuple(args[3])
    kind, key, numel = storage
    dt = _STORAGE_DTYPES.get(kind)
    if dt is None:
        msg = f"unsupported tensor storage {kind}"
        raise CheckpointFormatError(msg)
    raw = np.frombuffer(zf.read(f"{prefix}data/{key}"), dtype=dt)
    if raw.size != numel:
        msg = f"storage {key}: {raw.size} elements, record says {numel}"
        raise CheckpointFormatError(msg)
    # the view's geometry comes from the (untrusted) file: every element it
    # addresses must lie inside the storage before as_strided, which checks nothing
    if len(size) != len(stride) or offset < 0 or any(s < 0 for s in size) or any(s < 0 for s in stride):
        msg = f"storage {key}: invalid view (offset {offset}, size {size}, stride {stride})"
        raise CheckpointFormatError(msg)
    n_elem = int(np.prod(size, dtype=np.int64)) if size else 1
    last = offset + sum((n - 1) * s for n, s in zip(size, stride)) if n_elem else offset - 1
    if last >= raw.size:
        msg = f"storage {key}: view (offset {offset}, size {size}, stride {stride}) reaches element {last} of {raw.size}"
        raise CheckpointFormatError(msg)
    if not n_elem:
        return torch.from_numpy(np.zeros(size, dtype=dt))
    arr = np.lib.stride_tricks.as_strided(raw[offset:], shape=size, strides=tuple(s * raw.itemsize for s in stride)) if size else raw[offset : offset + 1].reshape(())
    return torch.from_numpy(np.array(arr, copy=True))


def read_inert(path):
    """The checkpoint's top-level object as inert data (see the module docstring)."""
    zf = zipfile.ZipFile(path)
    pkls = [n for n in zf.namelist() if n.endswith("data.pkl")]
    if len(pkls) != 1:
        msg = f"{path}: not a torch zip checkpoint (data.pkl entries: {len(pkls)})"
        raise CheckpointFormatError(msg)
    prefix = pkls[0][: -len("data.pkl")]
    stack, memo = [], {}

    def pop_mark():
        i = len(stack) - 1
        while stack[i] is not _MARK:
            i -= 1
        items = stack[i + 1 :]
        del stack[i:]
        return items

    def call(fn, args):
        if isinstance(fn, GlobalRef):
            if (fn.module, fn.name) == ("torch._utils", "_rebuild_tensor_v2"):
                return _rebuild_tensor(zf, prefix, args)
            if (fn.module, fn.name) == ("collections", "OrderedDict"):
                return dict(args[0]) if args else {}
            if (fn.module, fn.name) in (("builtins", "set"), ("__builtin__", "set")):
                return set(args[0]) if args else set()
            if (fn.module, fn.name) == ("_codecs", "encode") and len(args) == 2 and isinstance(args[0], str) and args[1] == "latin1":
                return args[0].encode("latin1")  # a bytes literal of protocol 2
            if (fn.module, fn.name) == ("numpy", "dtype") and args and isinstance(args[0], str) and args[0] in _NP_CODES:
                return np.dtype(args[0])
            if fn.module in ("numpy.core.multiarray", "numpy._core.multiarray") and fn.name == "scalar" and len(args) == 2 and isinstance(args[0], np.dtype) and isinstance(args[1], bytes):
                return np.frombuffer(args[1], dtype=args[0])[0]
            if fn.module in ("numpy.core.multiarray", "numpy._core.multiarray") and fn.name == "_reconstruct":
                return _NdArray()  # filled by BUILD
            if (fn.module, fn.name) == ("copyreg", "_reconstructor") and args and isinstance(args[0], GlobalRef):
                return Obj(args[0])  # object.__new__(cls): the instance's class, its state follows (BUILD)
        return Obj(fn if isinstance(fn, GlobalRef) else GlobalRef("?", repr(fn)), tuple(args))

    for op, arg, _pos in pickletools.genops(zf.read(pkls[0])):
        n = op.name
        if n in ("PROTO", "FRAME"):
            continue
        if n == "STOP":
            break
        if n == "MARK":
            stack.append(_MARK)
        elif n in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[arg] = stack[-1]
        elif n == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif n in ("BINGET", "LONG_BINGET", "GET"):
            stack.append(memo[arg])
        elif n in ("BINUNICODE", "SHORT_BINUNICODE", "BINUNICODE8", "UNICODE", "BINSTRING", "SHORT_BINSTRING", "STRING"):
            stack.append(arg)
        elif n in ("BINBYTES", "SHORT_BINBYTES", "BINBYTES8"):
            stack.append(bytes(arg))
        elif n in ("BININT", "BININT1", "BININT2", "INT", "LONG", "LONG1", "LONG4", "BINFLOAT", "FLOAT"):
            stack.append(arg)
        elif n == "NONE":
            stack.append(None)
        elif n == "NEWTRUE":
            stack.append(True)
        elif n == "NEWFALSE":
            stack.append(False)
        elif n == "EMPTY_DICT":
            stack.append({})
        elif n == "EMPTY_LIST":
            stack.append([])
        elif n == "EMPTY_TUPLE":
            stack.append(())
        elif n == "EMPTY_SET":
            stack.append(set())
        elif n == "TUPLE":
            stack.append(tuple(pop_mark()))
        elif n in ("TUPLE1", "TUPLE2", "TUPLE3"):
            k = int(n[-1])
            t = tuple(stack[-k:])
            del stack[-k:]
            stack.append(t)
        elif n == "LIST":
            stack.append(list(pop_mark()))
        elif n == "DICT":
            items = pop_mark()
            stack.append(dict(zip(items[::2], items[1::2])))
        elif n == "APPEND":
            v = stack.pop()
            stack[-1].append(v)
        elif n == "APPENDS":
            items = pop_mark()
            stack[-1].extend(items)
        elif n == "SETITEM":
            v, k = stack.pop(), stack.pop()
            _setitem(stack[-1], k, v)
        elif n == "SETITEMS":
            items = pop_mark()
            for k, v in zip(items[::2], items[1::2]):
                _setitem(stack[-1], k, v)
        elif n == "ADDITEMS":
            items = pop_mark()
            stack[-1].update(items)
        elif n == "FROZENSET":
            stack.append(frozenset(pop_mark()))
        elif n == "GLOBAL":
            mod, name = arg.split(" ", 1)
            stack.append(GlobalRef(mod, name))
        elif n == "STACK_GLOBAL":
            name, mod = stack.pop(), stack.pop()
            stack.append(GlobalRef(mod, name))
        elif n == "REDUCE":
            args, fn = stack.pop(), stack.pop()
            stack.append(call(fn, args))
        elif n in ("NEWOBJ", "NEWOBJ_EX"):
            if n == "NEWOBJ_EX":
                stack.pop()  # kwargs
            args, cls = stack.pop(), stack.pop()
            stack.append(Obj(cls, tuple(args)))
        elif n == "BUILD":
            st = stack.pop()
            obj = stack[-1]
            if isinstance(obj, Obj):
                obj.state = st
            elif isinstance(obj, np.dtype):
                if isinstance(st, tuple) and len(st) > 1 and st[1] == ">":
                    msg = "big-endian numpy data"
                    raise CheckpointFormatError(msg)
            elif isinstance(obj, _NdArray):  # (version, shape, dtype, fortran, raw bytes)
                _ver, shape, dt, fortran, raw = st
                if not isinstance(dt, np.dtype) or not isinstance(raw, bytes):
                    msg = "numpy array of objects"
                    raise CheckpointFormatError(msg)
                obj.value = np.frombuffer(raw, dtype=dt).reshape(shape, order="F" if fortran else "C").copy()
            elif isinstance(obj, (torch.Tensor, dict)):
                pass  # attributes of a tensor (_backward_hooks) or an OrderedDict (state_dict _metadata): ignored
            else:
                msg = f"BUILD on {type(obj).__name__}"
                raise CheckpointFormatError(msg)
        elif n == "BINPERSID":
            pid = stack.pop()  # ('storage', GlobalRef(torch, FloatStorage), key, location, numel)
            if not (isinstance(pid, tuple) and pid and pid[0] == "storage"):
                msg = f"unknown persistent id {pid!r}"
                raise CheckpointFormatError(msg)
            kind = pid[1].name if isinstance(pid[1], GlobalRef) else str(pid[1])
            stack.append((kind, pid[2], int(pid[4])))
        elif n == "POP":
            stack.pop()
        elif n == "POP_MARK":
            pop_mark()
        elif n == "DUP":
            stack.append(stack[-1])
        else:
            msg = f"pickle opcode {n} not handled by the inert reader"
            raise CheckpointFormatError(msg)
    if len(stack) != 1:
        msg = f"malformed pickle (stack depth {len(stack)} at STOP)"
        raise CheckpointFormatError(msg)
    return _finish(stack[0])


def _finish(v):
    """Replace the array placeholders by their arrays (recursively)."""
    if isinstance(v, _NdArray):
        return v.value
    if isinstance(v, dict):
        return {k: _finish(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_finish(x) for x in v]
    if isinstance(v, tuple):
        return tuple(_finish(x) for x in v)
    return v


def _setitem(obj, k, v):
    if isinstance(obj, dict):
        obj[k] = v
    elif isinstance(obj, Obj):
        obj.items[k] = v
    else:
        msg = f"SETITEM on {type(obj).__name__}"
        raise CheckpointFormatError(msg)


def class_name(v):
    """'Adam' for an optimizer instance / class reference, 'CrossEntropyLoss' for a loss, ...; strings pass through."""
    while isinstance(v, Obj):
        if v.cls == GlobalRef("dill._dill", "_create_type") and len(v.args) > 1 and isinstance(v.args[1], str):
            return v.args[1]  # a class pickled by dill: (metaclass, name, bases, namespace) -- its name only
        v = v.cls
    if isinstance(v, GlobalRef):
        return v.name
    return v


def load_checkpoint(path):
    """A DeepRank2 checkpoint dict: ``torch.load(weights_only=True)`` when the
    file allows it (this package's own checkpoints), else the inert reader
    (reference checkpoints), with class-valued entries (``data_type``,
    ``optimizer``, ``lossfunction``) reduced to their class names."""
    try:
        return torch.load(path, map_location="cpu", weights_only=True)
    except Exception:  # noqa: BLE001  (weights_only refusal or an unpicklable global)
        pass
    state = read_inert(path)
    if not isinstance(state, dict):
        msg = f"{path}: the checkpoint's top level is {type(state).__name__}, not a dict"
        raise CheckpointFormatError(msg)
    for k in ("data_type", "optimizer", "lossfunction"):
        if k in state:
            state[k] = class_name(state[k])
    return state


# ---- feature transforms stored as lambda source strings --------------------
# The reference saves each features_transform entry's lambda as its source text
# (trainer.py:_save_model via inspect) and eval()s it on load (dataset.py:118-122).
# Here the text is parsed with ast and interpreted: one-argument lambdas over
# arithmetic, numeric constants and a fixed set of numpy functions; anything
# else is refused.

import ast  # noqa: E402
import operator  # noqa: E402

_NP_FUNCS = {
    name: getattr(np, name)
    for name in ("log", "log2", "log10", "log1p", "exp", "expm1", "sqrt", "cbrt", "abs", "absolute", "tanh", "sinh", "cosh", "arcsinh", "sign", "square", "reciprocal", "clip", "maximum", "minimum", "power")
}
_BINOPS = {ast.Add: operator.add, ast.Sub: operator.sub, ast.Mult: operator.mul, ast.Div: operator.truediv, ast.Pow: operator.pow, ast.FloorDiv: operator.floordiv, ast.Mod: operator.mod}
_UNOPS = {ast.USub: operator.neg, ast.UAdd: operator.pos}


class TransformSourceError(ValueError):
    pass


def _compile_node(node, arg):
    if isinstance(node, ast.Name):
        if node.id != arg:
            msg = f"unknown name {node.id!r}"
            raise TransformSourceError(msg)
        return lambda t: t
    if isinstance(node, ast.Constant) and isinstance(node.value, (int, float)) and not isinstance(node.value, bool):
        v = node.value
        return lambda _t: v
    if isinstance(node, ast.BinOp) and type(node.op) in _BINOPS:
        f, a, b = _BINOPS[type(node.op)], _compile_node(node.left, arg), _compile_node(node.right, arg)
        return lambda t: f(a(t), b(t))
    if isinstance(node, ast.UnaryOp) and type(node.op) in _UNOPS:
        f, a = _UNOPS[type(node.op)], _compile_node(node.operand, arg)
        return lambda t: f(a(t))
    if isinstance(node, ast.Call) and not node.keywords and isinstance(node.func, ast.Attribute) and isinstance(node.func.value, ast.Name) and node.func.value.id in ("np", "numpy") and node.func.attr in _NP_FUNCS:
        f = _NP_FUNCS[node.func.attr]
        parts = [_compile_node(a, arg) for a in node.args]
        return lambda t: f(*(p(t) for p in parts))
    msg = f"unsupported expression {ast.dump(node)[:80]}"
    raise TransformSourceError(msg)


def transform_from_source(src: str):
    """A callable for a stored ``lambda t: ...`` transform (see above), without eval."""
    text = src.strip()
    try:
        tree = ast.parse(text, mode="eval")
    except SyntaxError as e:
        msg = f"transform {src!r} is not an expression"
        raise TransformSourceError(msg) from e
    lam = tree.body
    if not isinstance(lam, ast.Lambda) or len(lam.args.args) != 1 or lam.args.vararg or lam.args.kwarg or lam.args.kwonlyargs or lam.args.defaults:
        msg = f"transform {src!r} is not a one-argument lambda"
        raise TransformSourceError(msg)
    body = _compile_node(lam.body, lam.args.args[0].arg)

    def transform(t):
        return body(t)

    transform.source = text
    return transform
