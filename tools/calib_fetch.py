"""Runs tools/calib_fetch.hip's four access patterns over 1 GiB each (3 launches
per pattern, after the buffer has been written, so the Infinity Cache holds at
most a quarter of it).  Under `rocprofv3 --kernel-trace --pmc FETCH_SIZE` (and a
second pass with WRITE_SIZE) the counters per dispatch divided by 1 GiB are the
correction factors for each access width (tools/pmc_traffic.py).

  python tools/calib_fetch.py build     # here (hipcc, no GPU)
  python tools/calib_fetch.py           # on the GPU box
"""
import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libcalib_fetch.so")
BYTES = 1 << 30


def build():
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared",
                           os.path.join(HERE, "calib_fetch.hip"), "-o", SO])


def main():
    import torch
    lib = ctypes.CDLL(SO)
    lib.calib_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    buf = torch.ones(BYTES // 4, dtype=torch.float32, device="cuda:0")
    sink = torch.zeros(1, device="cuda:0")
    torch.cuda.synchronize()
    for kind in (0, 1, 2, 3):
        for _ in range(3):
            rc = lib.calib_run(kind, buf.data_ptr(), BYTES, sink.data_ptr())
            assert rc == 0, rc
    print("calib ok: kinds 0 (16-B loads), 1 (8-B granule loads), 2 (8-B granule stores, 32-B lane stride), "
          "3 (8-B granule stores, lane-consecutive), "
          f"{BYTES} B per launch")


if __name__ == "__main__":
    build() if sys.argv[1:] == ["build"] else main()
