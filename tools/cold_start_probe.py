import time, sys
t0=time.perf_counter()
sys.path.insert(0, "warmup-fir-filter_amd")
import numpy as np
t1=time.perf_counter()
import fir_hip
t2=time.perf_counter()
L=fir_hip.lib()
t3=time.perf_counter()
import ctypes
c=ctypes.c_int(0); L.fir_device_count(ctypes.byref(c))
t4=time.perf_counter()
fir_hip.fir1d_fixed_rows(np.zeros((2,64),np.uint8),[1,2,1])
t5=time.perf_counter()
fir_hip.fir1d_fixed_rows(np.zeros((2,64),np.uint8),[1,2,1])
t6=time.perf_counter()
fir_hip.fir1d_ideal_rows(np.zeros((2,64),np.uint8),[0.25,0.5,0.25])
t7=time.perf_counter()
b=fir_hip.host_empty(544<<20)
t8=time.perf_counter()
print(dict(numpy=t1-t0, import_fir_hip=t2-t1, lib_load=t3-t2, device_count=t4-t3, first_call=t5-t4, second_call=t6-t5, first_ideal=t7-t6, pinned_544MB=t8-t7))
