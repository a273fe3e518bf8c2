import ctypes, time, numpy as np, sys, os
sys.path.insert(0, os.getcwd())
from decds_amd._capi import lib, CODED_PIECE_BYTES as F
L=lib()
d=np.random.default_rng(1).integers(0,256,F,dtype=np.uint8)
out=ctypes.create_string_buffer(32)
L.decds_chunk_digest.argtypes=[ctypes.c_uint64,ctypes.c_uint64,ctypes.c_void_p,ctypes.c_size_t,ctypes.c_void_p]
for _ in range(3): L.decds_chunk_digest(1,2,d.ctypes.data,F,out)
t=time.perf_counter()
for _ in range(50): L.decds_chunk_digest(1,2,d.ctypes.data,F,out)
dt=(time.perf_counter()-t)/50
print("chunk digest 1 MiB: %.3f ms = %.2f GB/s"%(dt*1e3, F/dt/1e9))
big=np.random.default_rng(2).integers(0,256,256<<20,dtype=np.uint8)
for th in (1,4,16):
    t=time.perf_counter()
    for _ in range(3): L.decds_blake3_parallel(big.ctypes.data_as(ctypes.c_void_p), big.size, out, th)
    dt=(time.perf_counter()-t)/3
    print("blake3_parallel 256 MiB threads=%d: %.2f GB/s"%(th, big.size/dt/1e9))
