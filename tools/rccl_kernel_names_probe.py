"""Which kernels does a world-1 RCCL exchange launch, and does the bench's
trace classifier see them as RCCL?  Run under rocprofv3 --kernel-trace:

    rocprofv3 --kernel-trace -d gpurun_out/rk -o rk --output-format csv -- python tools/rccl_kernel_names_probe.py
    python tools/rccl_kernel_names_probe.py --classify gpurun_out/rk

The probe opens a one-rank communicator (bm_comm_init), runs bm_allgatherv
in its ncclAllGather and point-to-point forms and a bm_alltoallv, between
torch spin-kernel markers; --classify prints every kernel of the trace with
bench.kernel_class()."""
import ctypes
import glob
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def run():
    import torch
    from bolt_amd.mi355x import _lib
    torch.cuda.set_device(0)
    lib = _lib.load()
    uid = ctypes.create_string_buffer(_lib.COMM_ID_BYTES)
    _lib.check(lib.bm_comm_unique_id(uid, _lib.COMM_ID_BYTES), "bm_comm_unique_id")
    c = ctypes.c_void_p()
    _lib.check(lib.bm_comm_init(ctypes.byref(c), 1, uid, 0), "bm_comm_init")
    st = torch.cuda.current_stream().cuda_stream
    x = torch.randint(0, 255, (64 << 20,), dtype=torch.uint8, device="cuda")
    y = torch.empty_like(x)
    torch.cuda._sleep(1)
    _lib.check(lib.bm_allgatherv(c.value, x.data_ptr(), x.numel(), y.data_ptr(), _lib.i64_array([x.numel()]),
                                 _lib.i64_array([0]), st), "bm_allgatherv")
    torch.cuda._sleep(1)
    _lib.check(lib.bm_alltoallv(c.value, x.data_ptr(), _lib.i64_array([x.numel()]), _lib.i64_array([0]),
                                y.data_ptr(), _lib.i64_array([x.numel()]), _lib.i64_array([0]), st), "bm_alltoallv")
    torch.cuda._sleep(1)
    _lib.check(lib.bm_comm_wait(c.value, st, 60.0), "bm_comm_wait")
    assert torch.equal(x, y)
    _lib.check(lib.bm_comm_destroy(c.value), "bm_comm_destroy")
    print("probe ok")


def classify(d):
    import csv
    import bench
    for f in sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            print("%-8s %9.1f us  %s" % (bench.kernel_class(n), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3,
                                        n[:140]))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--classify":
        classify(sys.argv[2])
    else:
        run()
