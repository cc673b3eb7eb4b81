"""The 'mi355x' mode: BoltArrayMI355X, ChunkedArrayMI355X, ConstructMI355X.

Layout mirrors bolt/spark/ (array.py, chunk.py, construct.py, shapes.py) plus
the MI355X runtime pieces: _lib (ctypes C ABI), _ops (kernel launches),
context (devices and ranks), dist (RCCL exchanges), plan (host planning).
"""
