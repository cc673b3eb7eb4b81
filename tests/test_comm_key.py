"""RCCL rendezvous keys of MI355XContext (context.py _comm_key): counted per
rank set, so ranks that open contexts over different subgroups in different
orders still read the unique id their own group's rank 0 wrote."""
from bolt_amd.mi355x.context import MI355XContext


def test_comm_key_per_rank_set(monkeypatch):
    monkeypatch.setattr(MI355XContext, "_ncomm", {})
    # process A: world, then subgroup {1, 2}; process B: subgroup {1, 2} only
    a_world = MI355XContext._comm_key(range(4))
    a_sub = MI355XContext._comm_key([1, 2])
    monkeypatch.setattr(MI355XContext, "_ncomm", {})
    b_sub = MI355XContext._comm_key((1, 2))
    assert a_sub == b_sub
    assert a_world != a_sub
    # a second communicator over the same ranks gets a fresh key
    assert MI355XContext._comm_key((1, 2)) != b_sub
