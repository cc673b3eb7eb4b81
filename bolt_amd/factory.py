"""Mode registry and router: bolt/factory.py with the 'mi355x' mode added.

Restates bolt/factory.py:4-83 with two fixes a drop-in needs:
  * ``mode=`` routing works (the reference tests ``mode not in constructors``
    against a list of tuples, factory.py:45-50, so every mode raised);
  * docstrings are built with ``inspect.signature`` (``inspect.getargspec``,
    factory.py:17, is gone from Python >= 3.11).
Routing without ``mode=`` is unchanged: the first constructor whose
``_argcheck`` accepts the arguments wins, local is the default.
"""
import inspect

from bolt_amd.mi355x.construct import ConstructMI355X
from bolt_amd.local import ConstructLocal

constructors = [
    ('local', ConstructLocal),
    ('mi355x', ConstructMI355X),
]


def _signature(func):
    try:
        return str(inspect.signature(func))
    except (TypeError, ValueError):  # pragma: no cover
        return "(...)"


def wrapped(f):
    """Append each mode's constructor signature to the routed docstring (factory.py:9-35)."""
    doc = (f.__doc__ or "") + "\n"
    for mode, constructor in constructors:
        method = getattr(constructor, f.__name__, None)
        if method is not None:
            doc += "    %s -> %s%s\n" % (mode, f.__name__, _signature(method))
    f.__doc__ = doc
    return f


def lookup(*args, **kwargs):
    """Pick the constructor for these arguments (factory.py:37-55)."""
    if 'mode' in kwargs:
        mode = kwargs['mode']
        table = dict(constructors)
        if mode not in table:
            raise ValueError('Mode %s not supported' % mode)
        del kwargs['mode']
        return table[mode]
    for mode, constructor in constructors:
        if constructor._argcheck(*args, **kwargs):
            return constructor
    return ConstructLocal


def _strip_mode(kwargs):
    kwargs = dict(kwargs)
    kwargs.pop('mode', None)
    return kwargs


@wrapped
def array(*args, **kwargs):
    """Create a bolt array."""
    return lookup(*args, **kwargs).dispatch('array', *args, **_strip_mode(kwargs))


@wrapped
def ones(*args, **kwargs):
    """Create a bolt array of ones."""
    return lookup(*args, **kwargs).dispatch('ones', *args, **_strip_mode(kwargs))


@wrapped
def zeros(*args, **kwargs):
    """Create a bolt array of zeros."""
    return lookup(*args, **kwargs).dispatch('zeros', *args, **_strip_mode(kwargs))


@wrapped
def concatenate(*args, **kwargs):
    """Join two bolt arrays (factory.py:78-83)."""
    return lookup(*args, **kwargs).dispatch('concatenate', *args, **_strip_mode(kwargs))
