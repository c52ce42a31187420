"""Can the 2-D CFAR (K3, VALU-bound) of one batch overlap the range / Doppler kernels (K1 / K2,
HBM-bound) of the next?  Config 5, 16 frames per batch, two handles on two HIP streams:
A = K1 + K2 only (cfar none), B = K3 only (fmcw_cfar over a map A produced).  Times A alone,
B alone, both one after the other on one stream, and both at once on two streams, for K3 grid
caps given on the command line (FMCW_GRID_CFAR, read at fmcw_create).

usage: python tools/overlap_lab.py [iters] [cap ...]     (cap 0 = the occupancy grid)
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fpga-fmcw-radar-processor_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fmcw import RadarCore, DeviceBuffer, synth  # noqa: E402

NF, NS, NC = 16, 8192, 1024


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    caps = [int(x) for x in sys.argv[2:]] or [0]
    torch.cuda.init()
    u = synth.frames(4, NS, NC, 1, "two_targets", seed=1234, dtype="f16")
    cube = np.ascontiguousarray(np.concatenate([u] * (NF // 4)))
    din = DeviceBuffer(cube.nbytes)
    din.upload(cube)
    map_a = DeviceBuffer(NF * NS * NC * 4)
    map_b = DeviceBuffer(NF * NS * NC * 4)
    cap = 1 << 20
    dd, dn = DeviceBuffer(cap * 16), DeviceBuffer(64)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    a = RadarCore(N_RANGE=NS, N_DOPPLER=NC, in_dtype="f16", cfar="none", max_frames=NF)
    a.enqueue(din, NF, rd_map=map_a)
    torch.cuda.synchronize()
    map_b.copy_from(map_a, NF * NS * NC * 4)
    torch.cuda.synchronize()

    def timed(fn):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(iters):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return 1e3 * float(np.median(ts))

    for c in caps:
        if c:
            os.environ["FMCW_GRID_CFAR"] = str(c)
        else:
            os.environ.pop("FMCW_GRID_CFAR", None)
        b = RadarCore(N_RANGE=NS, N_DOPPLER=NC, in_dtype="f16", cfar="os2d", max_frames=NF)
        ka = lambda st: a.enqueue(din, NF, rd_map=map_a, stream=st.cuda_stream)
        kb = lambda st: b.cfar(map_b, NF, dd, cap, dn, stream=st.cuda_stream)
        t_a = timed(lambda: ka(s1))
        t_b = timed(lambda: kb(s2))
        t_seq = timed(lambda: (ka(s1), kb(s1)))
        t_par = timed(lambda: (kb(s2), ka(s1)))
        t_par2 = timed(lambda: (ka(s1), kb(s2)))
        n = int(dn.download(np.uint32, (1,))[0])
        print(f"K3 grid cap {c or 'occupancy'}: A (K1+K2) {t_a:.3f} ms, B (K3) {t_b:.3f} ms, "
              f"sequential {t_seq:.3f} ms, concurrent K3-first {t_par:.3f} ms, K1-first {t_par2:.3f} ms, "
              f"dets {n}", flush=True)
        b.close()
    a.close()


if __name__ == "__main__":
    main()
