"""Non-executing reader for the reference's pickled code objects.

The reference stores its hypergraph-product codes as pickled ``bposd.hgp.hgp``
objects (``codes_lib/hgp_34_n225.pkl``, loaded by ``load_object`` at
``src/Simulators.py:69-71``).  Unpickling would import and call whatever the file
names, so this module never unpickles: it walks the opcode stream with
``pickletools.genops`` and interprets a small, closed subset of opcodes on a
private stack of plain tuples.  Globals are recorded as ``("global", module,
name)`` strings and are never imported or called; the only structures that are
turned into values are numpy ``_reconstruct``/``scalar`` payloads (raw bytes +
shape + dtype string) and Python scalars.  Any opcode outside the subset raises.
"""
from __future__ import annotations

import pickletools

import numpy as np

_MARK = object()


class UnsupportedPickle(ValueError):
    pass


def _interpret(data: bytes):
    stack: list = []
    memo: dict = {}
    for op, arg, _pos in pickletools.genops(data):
        name = op.name
        if name in ("PROTO", "FRAME"):
            continue
        if name == "STOP":
            break
        if name == "MARK":
            stack.append(_MARK)
        elif name in ("BININT", "BININT1", "BININT2", "LONG1", "LONG4", "INT", "LONG"):
            stack.append(int(arg))
        elif name in ("BINFLOAT", "FLOAT"):
            stack.append(float(arg))
        elif name in ("SHORT_BINUNICODE", "BINUNICODE", "BINUNICODE8", "UNICODE"):
            stack.append(str(arg))
        elif name in ("SHORT_BINBYTES", "BINBYTES", "BINBYTES8"):
            stack.append(bytes(arg))
        elif name == "NEWTRUE":
            stack.append(True)
        elif name == "NEWFALSE":
            stack.append(False)
        elif name == "NONE":
            stack.append(None)
        elif name == "EMPTY_TUPLE":
            stack.append(())
        elif name in ("TUPLE1", "TUPLE2", "TUPLE3"):
            k = int(name[-1])
            items = tuple(stack[-k:])
            del stack[-k:]
            stack.append(items)
        elif name == "TUPLE":
            i = len(stack) - 1 - stack[::-1].index(_MARK)
            items = tuple(stack[i + 1:])
            del stack[i:]
            stack.append(items)
        elif name == "EMPTY_DICT":
            stack.append({})
        elif name == "EMPTY_LIST":
            stack.append([])
        elif name == "SETITEM":
            v = stack.pop()
            k = stack.pop()
            stack[-1][k] = v
        elif name == "SETITEMS":
            i = len(stack) - 1 - stack[::-1].index(_MARK)
            items = stack[i + 1:]
            del stack[i:]
            d = stack[-1]
            for k, v in zip(items[0::2], items[1::2]):
                d[k] = v
        elif name == "APPEND":
            v = stack.pop()
            stack[-1].append(v)
        elif name == "APPENDS":
            i = len(stack) - 1 - stack[::-1].index(_MARK)
            items = stack[i + 1:]
            del stack[i:]
            stack[-1].extend(items)
        elif name == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif name in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[int(arg)] = stack[-1]
        elif name in ("BINGET", "LONG_BINGET", "GET"):
            stack.append(memo[int(arg)])
        elif name == "STACK_GLOBAL":
            nm = stack.pop()
            mod = stack.pop()
            stack.append(("global", str(mod), str(nm)))
        elif name == "GLOBAL":
            mod, nm = str(arg).split(" ", 1)
            stack.append(("global", mod, nm))
        elif name == "REDUCE":
            args = stack.pop()
            fn = stack.pop()
            stack.append(["reduce", fn, args, None])
        elif name == "NEWOBJ":
            args = stack.pop()
            cls = stack.pop()
            stack.append(["newobj", cls, args, None])
        elif name == "BUILD":
            state = stack.pop()
            obj = stack[-1]
            if not isinstance(obj, list) or len(obj) != 4:
                raise UnsupportedPickle("BUILD on unsupported object")
            obj[3] = state
        else:
            raise UnsupportedPickle(f"opcode {name} not supported by the safe reader")
    if len(stack) != 1:
        raise UnsupportedPickle("malformed pickle stream")
    return stack[0]


def _dtype_of(obj) -> np.dtype:
    # ["reduce", ("global","numpy","dtype"), ("f8", False, True), state]
    if not (isinstance(obj, list) and obj[0] == "reduce" and obj[1][2] == "dtype"):
        raise UnsupportedPickle("unexpected dtype encoding")
    code = obj[2][0]
    state = obj[3]
    order = state[1] if state and len(state) > 1 and state[1] in "<>|=" else "<"
    return np.dtype(code).newbyteorder(order if order != "|" else "=")


def _value(obj):
    if isinstance(obj, list) and obj[0] == "reduce":
        fn = obj[1]
        if fn[0] == "global" and fn[2] == "_reconstruct":
            st = obj[3]  # (version, shape, dtype, is_fortran, rawbytes)
            _ver, shape, dt, fortran, raw = st
            dtype = _dtype_of(dt)
            arr = np.frombuffer(raw, dtype=dtype)
            return arr.reshape(shape, order="F" if fortran else "C").copy()
        if fn[0] == "global" and fn[2] == "scalar":
            dt, raw = obj[2]
            return np.frombuffer(raw, dtype=_dtype_of(dt))[0].item()
        return None
    if isinstance(obj, (int, float, str, bool)) or obj is None:
        return obj
    return None


def load_pickled_code_arrays(path: str) -> dict:
    """Return the attribute dict of a pickled ``bposd.hgp.hgp``/``css_code``.

    Only numpy arrays and Python/numpy scalars are materialised; anything else
    maps to ``None``.  The class named in the file is reported under
    ``"__class__"`` as a string and never imported.
    """
    with open(path, "rb") as f:
        data = f.read()
    root = _interpret(data)
    if not (isinstance(root, list) and root[0] in ("newobj", "reduce")):
        raise UnsupportedPickle("top-level object is not a class instance")
    state = root[3]
    if not isinstance(state, dict):
        raise UnsupportedPickle("instance state is not a dict")
    out = {k: _value(v) for k, v in state.items()}
    cls = root[1]
    out["__class__"] = f"{cls[1]}.{cls[2]}" if cls[0] == "global" else "?"
    return out
