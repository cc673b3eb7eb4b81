"""User-function plumbing of the mi355x mode (map / map_generic / stack / filter).

bolt applies numpy functions to records on Spark executors (chunk.py:349-432,
stack.py:80-139, array.py:125-241).  Here records live in HBM, so the user
function receives torch tensors on the array's device and should be written
with torch operations (numpy-style spellings such as ``x.sum(axis=1,
keepdims=True)`` work on tensors); a function that returns an ndarray has it
moved to the device.  Record-wise functions are vectorised with torch.func.vmap
over a batch of records or chunks (one launch per op for the whole batch); a
function vmap cannot trace (data-dependent control flow, .item(), host
numpy) is applied record by record, still on the device.
"""
import numpy as np

_NP2TORCH = None


def torch_dtype(dtype):
    global _NP2TORCH
    import torch
    if _NP2TORCH is None:
        _NP2TORCH = {np.dtype(k): v for k, v in [
            (np.bool_, torch.bool), (np.uint8, torch.uint8), (np.int8, torch.int8),
            (np.uint16, torch.uint16), (np.int16, torch.int16), (np.uint32, torch.uint32),
            (np.int32, torch.int32), (np.uint64, torch.uint64), (np.int64, torch.int64),
            (np.float16, torch.float16), (np.float32, torch.float32), (np.float64, torch.float64),
            (np.complex64, torch.complex64), (np.complex128, torch.complex128)]}
    try:
        return _NP2TORCH[np.dtype(dtype)]
    except KeyError:
        raise NotImplementedError("dtype %s has no device representation" % np.dtype(dtype))


def numpy_dtype(tdtype):
    torch_dtype(np.float32)  # builds the table
    for k, v in _NP2TORCH.items():
        if v == tdtype:
            return k
    raise NotImplementedError("torch dtype %s has no numpy counterpart" % tdtype)


def user_fn(func):
    """``func`` as the mode hands it records: torch has no arithmetic for
    uint16 / uint32 (2.10: add, comparisons, max, neg raise NotImplementedError),
    where the reference's numpy records compute in the fixed-width type.  Such
    tensors reach ``func`` widened to int64 (every value exact), and the
    result's dtype is put back to numpy's:
      * when ``func`` also runs on a numpy record of the same shape and dtype
        (a zero record, once per shape; most record functions do), the result
        takes the dtype numpy gives -- uint32 for ``v * 2`` (wrap-around),
        uint64 for ``v.sum()``, int64 for an explicit ``astype(int64)``; a
        torch-only function that runs on an unwidened zero record (an
        explicit ``v.to(torch.int64)``) keeps torch's dtype for it;
      * otherwise a result of the record's own shape in the widened type is
        elementwise and comes back in the record type (numpy's wrap-around for
        + - * & | ^ <<, exact for comparisons, min / max and //); any other
        result keeps the widened type (exact).
    Keys (``with_keys`` pairs) pass through; other dtypes are untouched."""
    import torch
    wide = {torch.uint16: torch.int64, torch.uint32: torch.int64}
    probes = {}

    def widen(a):
        if isinstance(a, torch.Tensor) and a.dtype in wide:
            return a.to(wide[a.dtype]), a.dtype
        if isinstance(a, tuple) and not isinstance(a, KeyTuple):  # a (key, value) pair
            parts = [widen(x) for x in a]
            orig = next((o for _, o in parts if o is not None), None)
            return type(a)(x for x, _ in parts) if type(a) is tuple else a, orig
        return a, None

    def numpy_dtype_of(shape, orig):
        """The result dtype of func on a zero record of the record's own dtype:
        numpy's where func takes ndarrays, else torch's where func needs no
        arithmetic torch lacks (an explicit cast, a view), else None."""
        key = (tuple(shape), orig)
        if key not in probes:
            probes[key] = None
            try:
                with np.errstate(all="ignore"):
                    r = func(np.zeros(tuple(shape), dtype=numpy_dtype(orig)))
                if isinstance(r, (np.ndarray, np.generic)):
                    probes[key] = np.asarray(r).dtype
            except Exception:  # a torch-only function
                pass
            if probes[key] is None:
                try:
                    r = func(torch.zeros(tuple(shape), dtype=orig))
                    if isinstance(r, torch.Tensor):
                        probes[key] = numpy_dtype(r.dtype)
                except Exception:  # needs the widened arithmetic
                    pass
        return probes[key]

    def record_shape(a):
        if isinstance(a, torch.Tensor):
            return tuple(a.shape)
        if isinstance(a, tuple) and not isinstance(a, KeyTuple):
            return next((s for s in map(record_shape, a) if s is not None), None)
        return None

    def wrapped(*args):
        new, orig = [], None
        for a in args:
            w, o = widen(a)
            new.append(w)
            orig = orig or o
        out = func(*new)
        if orig is None or not isinstance(out, torch.Tensor) or out.dtype != wide[orig]:
            return out
        if len(args) == 1 and isinstance(args[0], torch.Tensor):
            want = numpy_dtype_of(args[0].shape, orig)
            if want is not None:
                return out if want == np.dtype(np.int64) else out.to(torch_dtype(want))
        # not numpy-callable: elementwise results return to the record type
        return out.to(orig) if tuple(out.shape) == record_shape(tuple(args)) else out
    return wrapped


def view(buf, shape, dtype):
    """A uint8 buffer seen as a tensor of ``dtype`` and ``shape`` (no copy)."""
    shape = tuple(int(s) for s in shape)
    if buf.numel() == 0:
        import torch
        return torch.empty(shape, dtype=torch_dtype(dtype), device=buf.device)
    return buf.view(torch_dtype(dtype)).reshape(shape)


def as_bytes(t):
    """A contiguous tensor's bytes as a flat uint8 tensor."""
    import torch
    t = t.contiguous()
    if t.dtype == torch.bool:
        t = t.view(torch.uint8)
    return t.reshape(-1).view(torch.uint8) if t.numel() else torch.empty(0, dtype=torch.uint8, device=t.device)


def to_device(out, device):
    """A user function's result as a tensor on ``device`` (ndarrays / scalars are moved)."""
    import torch
    if isinstance(out, torch.Tensor):
        return out if out.device == device else out.to(device)
    return torch.as_tensor(np.asarray(out), device=device)


def random_like(shape, dtype, device):
    """randn(*shape).astype(dtype) on the device -- the probe the reference
    feeds a function to learn its output shape (chunk.py:373-375, array.py:161)."""
    import torch
    r = torch.randn(tuple(int(s) for s in shape), dtype=torch.float64, device=device)
    dt = np.dtype(dtype)
    if dt.kind in "iub":
        r = r.trunc()
    return r.to(torch_dtype(dt))


def apply_batched(func, batch):
    """stack([func(batch[i]) for i]) -- vmapped when the function allows it."""
    import torch
    if batch.shape[0] == 0:
        return None
    try:
        from torch.func import vmap
        out = vmap(func)(batch)
        if isinstance(out, torch.Tensor):
            return out
    except Exception:
        pass
    outs = [to_device(func(batch[i]), batch.device) for i in range(batch.shape[0])]
    shapes = set(tuple(o.shape) for o in outs)
    if len(shapes) != 1:
        raise Exception("Map operation did not produce values of uniform shape.")
    return torch.stack(outs)


def apply_pairs(func, a, b):
    """stack([func(a[i], b[i]) for i]) -- a user reduce function over record
    pairs, vmapped when the function allows it (else one pair at a time)."""
    import torch
    if a.shape[0] == 0:
        try:
            from torch.func import vmap
            out = vmap(func)(a, b)
            if isinstance(out, torch.Tensor):
                return out
        except Exception:
            pass
        z = torch.zeros((1,) + tuple(a.shape[1:]), dtype=a.dtype, device=a.device)
        return to_device(func(z[0], z[0]), a.device)[None][:0]
    try:
        from torch.func import vmap
        out = vmap(func)(a, b)
        if isinstance(out, torch.Tensor) and out.shape[0] == a.shape[0]:
            return out
    except Exception:
        pass
    outs = [to_device(func(a[i], b[i]), a.device) for i in range(a.shape[0])]
    return torch.stack(outs)


class KeyTuple(tuple):
    """A record key handed to a ``with_keys`` user function: a plain tuple of
    ints (indexable, hashable) that, like a tuple meeting a numpy array in
    the reference (array.py:125-191 passes (key, ndarray) pairs), combines
    arithmetically with a device tensor: ``k + v`` adds the key broadcast
    against the value instead of raising tuple's concatenation TypeError."""

    def _t(self, other):
        import torch
        return torch.as_tensor(tuple(self), device=other.device)

    def _op(name, reflected=False):
        def f(self, other):
            import torch
            if isinstance(other, torch.Tensor):
                a, b = (other, self._t(other)) if reflected else (self._t(other), other)
                return getattr(a, name)(b)
            return getattr(super(KeyTuple, self), "__r%s__" % name[2:-2] if reflected else name,
                           lambda o: NotImplemented)(other)
        return f

    __add__ = _op("__add__")
    __radd__ = _op("__add__", reflected=True)
    __sub__ = _op("__sub__")
    __rsub__ = _op("__sub__", reflected=True)
    __mul__ = _op("__mul__")
    __rmul__ = _op("__mul__", reflected=True)
    __truediv__ = _op("__truediv__")
    __rtruediv__ = _op("__truediv__", reflected=True)
    del _op
