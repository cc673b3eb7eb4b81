"""Routing through the REFERENCE's factory once the mi355x mode is registered
(run by tests/test_reference_dropin.py under dropin_plugin, never directly)."""
import numpy as np

import bolt
import bolt.base
import bolt.factory
import bolt.local.array


def test_lookup_routes_to_mi355x(sc):
    from bolt_amd.mi355x.construct import ConstructMI355X
    from bolt_amd.mi355x.array import BoltArrayMI355X
    x = np.arange(24).reshape(2, 3, 4)
    assert bolt.factory.lookup(x, sc) is ConstructMI355X
    assert bolt.factory.lookup(x, context=sc) is ConstructMI355X
    b = bolt.array(x, sc, axis=(0, 1))
    assert isinstance(b, BoltArrayMI355X) and isinstance(b, bolt.base.BoltArray)
    assert b.mode == "mi355x" and b.split == 2
    assert bolt.factory.lookup(b) is ConstructMI355X
    assert np.array_equal(b.toarray(), x)
    # mode= (the fixed lookup) and keyword context
    c = bolt.array(x, mode="mi355x", context=sc)
    assert isinstance(c, BoltArrayMI355X) and np.array_equal(c.toarray(), x)
    # local stays local
    assert isinstance(bolt.array(x), bolt.local.array.BoltArrayLocal)
    assert isinstance(bolt.array(x, mode="local"), bolt.local.array.BoltArrayLocal)


def test_ones_zeros_concatenate(sc):
    from bolt_amd.mi355x.array import BoltArrayMI355X
    o = bolt.ones((3, 4), sc, dtype=np.int32)
    z = bolt.zeros((3, 4), context=sc)
    assert isinstance(o, BoltArrayMI355X) and np.array_equal(o.toarray(), np.ones((3, 4), np.int32))
    assert np.array_equal(z.toarray(), np.zeros((3, 4)))
    j = bolt.concatenate((o, np.ones((2, 4), np.int32)), axis=0)
    assert isinstance(j, BoltArrayMI355X) and j.shape == (5, 4)


def test_statistics_are_bolt_local(sc):
    x = (np.arange(60) % 7).reshape(3, 4, 5).astype(np.float64)
    b = bolt.array(x, sc)
    m = b.mean(axis=0)
    assert isinstance(m, bolt.local.array.BoltArrayLocal)
    assert np.allclose(m, x.mean(0))
    assert np.isclose(b.std(), x.std())
