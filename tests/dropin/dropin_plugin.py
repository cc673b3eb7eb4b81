"""pytest plugin: run the REFERENCE's own Spark-mode tests against the mi355x mode.

Loaded only by tests/test_reference_dropin.py, in a child process, in the build
container (it imports /root/reference; nothing here travels to the GPU box).
It applies INTEGRATION.md section 2 to the reference bolt in-process:

  * bolt_amd/base.py, bolt_amd/local.py and bolt_amd/construct.py are dropped
    in favour of bolt.base, bolt.local and bolt.construct (so BoltArrayMI355X
    IS a bolt.base.BoltArray and statistics return bolt's own BoltArrayLocal);
  * ('mi355x', ConstructMI355X) is appended to bolt.factory.constructors,
    bolt.factory.lookup gets the mode= fix (bolt/factory.py:37-56) and the
    routed array/ones/zeros/concatenate stop forwarding `mode` (:58-83);

and provides the `sc` fixture the reference tests take (test/conftest.py:11-16)
as an MI355XContext on the CPU test executor (tests/cpu_backend.py), so
`array(x, sc)` routes through the reference's own factory.lookup ->
ConstructMI355X._argcheck -> ConstructBase.dispatch (bolt/construct.py:3-8).
"""
import collections
import collections.abc
import sys
import types

import pytest

collections.Iterable = collections.abc.Iterable  # bolt/utils.py:3 on Python >= 3.10

import bolt  # noqa: E402  (the reference, from PYTHONPATH)
import bolt.base  # noqa: E402
import bolt.construct  # noqa: E402
import bolt.factory  # noqa: E402
import bolt.local.array  # noqa: E402
import bolt.local.construct  # noqa: E402

# drop bolt_amd's stand-ins for bolt's own modules
_local = types.ModuleType("bolt_amd.local")
_local.BoltArrayLocal = bolt.local.array.BoltArrayLocal
_local.ConstructLocal = bolt.local.construct.ConstructLocal
sys.modules["bolt_amd.base"] = bolt.base
sys.modules["bolt_amd.construct"] = bolt.construct
sys.modules["bolt_amd.local"] = _local

import bolt_amd  # noqa: E402
from bolt_amd.mi355x.array import BoltArrayMI355X  # noqa: E402
from bolt_amd.mi355x.construct import ConstructMI355X  # noqa: E402
from bolt_amd.mi355x.context import MI355XContext  # noqa: E402

assert issubclass(BoltArrayMI355X, bolt.base.BoltArray)
assert issubclass(ConstructMI355X, bolt.construct.ConstructBase)

# the factory patch
if ("mi355x", ConstructMI355X) not in bolt.factory.constructors:
    bolt.factory.constructors.append(("mi355x", ConstructMI355X))


def _lookup(*args, **kwargs):
    """bolt/factory.py:37-56 with the mode= branch fixed (a dict lookup)."""
    if "mode" in kwargs:
        table = dict(bolt.factory.constructors)
        mode = kwargs["mode"]
        if mode not in table:
            raise ValueError("Mode %s not supported" % mode)
        del kwargs["mode"]
        return table[mode]
    for mode, constructor in bolt.factory.constructors:
        if constructor._argcheck(*args, **kwargs):
            return constructor
    return bolt.local.construct.ConstructLocal


bolt.factory.lookup = _lookup


def _routed(name):
    """bolt/factory.py:58-83 with `mode` kept out of the constructor call (the
    reference forwards it to dispatch, so even a fixed lookup would raise a
    TypeError in ConstructLocal / ConstructSpark / ConstructMI355X)."""
    def f(*args, **kwargs):
        constructor = bolt.factory.lookup(*args, **kwargs)
        kwargs.pop("mode", None)
        return constructor.dispatch(name, *args, **kwargs)
    f.__name__ = name
    f.__doc__ = getattr(bolt.factory, name).__doc__
    return f


for _name in ("array", "ones", "zeros", "concatenate"):
    setattr(bolt.factory, _name, _routed(_name))
    setattr(bolt, _name, getattr(bolt.factory, _name))


@pytest.fixture(scope="session")
def sc():
    import cpu_backend
    cpu_backend.install()
    return MI355XContext(device="cpu")
