"""Argument coercion and validation helpers of the bolt API surface.

Same names, argument meaning and error behaviour as the reference's
``bolt/utils.py`` (cited per function) so that ``bolt_amd`` raises what bolt
raises.  Pure host logic; no device work happens here.
"""
from collections.abc import Iterable

import numpy as np


def tupleize(arg):
    """Coerce singletons, lists and ndarrays to tuples (bolt/utils.py:5-23)."""
    if arg is None:
        return None
    if not isinstance(arg, (tuple, list, np.ndarray, Iterable)):
        return (arg,)
    if isinstance(arg, (list, np.ndarray)):
        return tuple(arg)
    if isinstance(arg, Iterable) and not isinstance(arg, str):
        return tuple(arg)
    return arg


def argpack(args):
    """Coerce an argument list to a tuple: ((a,b),) or (a,b) -> (a,b) (bolt/utils.py:25-40)."""
    if isinstance(args[0], (tuple, list, np.ndarray)):
        return tupleize(args[0])
    if isinstance(args[0], Iterable) and not isinstance(args[0], str):
        return tupleize(list(args[0]))
    return tuple(args)


def inshape(shape, axes):
    """ValueError unless every axis is inside ``shape`` (bolt/utils.py:42-56)."""
    valid = all((axis < len(shape)) and (axis >= 0) for axis in axes)
    if not valid:
        raise ValueError("axes not valid for an ndarray of shape: %s" % str(shape))


def allclose(a, b):
    """Shape equality plus numpy.allclose (bolt/utils.py:58-71; the reference tests' oracle)."""
    return (a.shape == b.shape) and np.allclose(a, b)


def slicify(slc, dim):
    """A slice with explicit start/stop/step inside [0, dim] (bolt/utils.py:105-147).

    Start and stop are made non-negative; a negative step that runs past the
    front keeps stop = -1 (the one negative value, handled by the caller);
    an int i becomes slice(i, i+1, 1).
    """
    if isinstance(slc, slice):
        start = 0 if slc.start is None else slc.start
        stop = dim if slc.stop is None else slc.stop
        step = 1 if slc.step is None else slc.step
        if start < 0:
            start += dim
        if stop < 0:
            stop += dim
        if step > 0:
            if start < 0:
                start = 0
            if stop > dim:
                stop = dim
        else:
            if stop < 0:
                stop = -1
            if start > dim:
                start = dim - 1
        return slice(start, stop, step)
    elif isinstance(slc, int):
        if slc < 0:
            slc += dim
        return slice(slc, slc + 1, 1)
    else:
        raise ValueError("Type for slice %s not recongized" % type(slc))


def istransposeable(new, old):
    """Validate a proposed permutation: length, repeats, bounds (bolt/utils.py:149-172)."""
    new, old = tupleize(new), tupleize(old)
    if not len(new) == len(old):
        raise ValueError("Axes do not match axes of keys")
    if not len(set(new)) == len(set(old)):
        raise ValueError("Repeated axes")
    if any(n < 0 for n in new) or max(new) > len(old) - 1:
        raise ValueError("Invalid axes")


def isreshapeable(new, old):
    """ValueError unless the total size is unchanged (bolt/utils.py:174-191)."""
    new, old = tupleize(new), tupleize(old)
    if not np.prod(new) == np.prod(old):
        raise ValueError("Total size of new keys must remain unchanged")
