import sys, time, torch, numpy as np
sys.path.insert(0,'spark-timeseries_amd')
from sparkts import _native
_native.ensure_device(0); lib=_native.lib()
S,T=1_000_000,390
x=torch.empty((S,T),dtype=torch.float64,device='cuda'); sp=torch.cuda.current_stream().cuda_stream
assert lib.sts_gen_panel(x.data_ptr(),0,S,T,T,6,0.0,sp)==0
sm=torch.full((S,),0.5,dtype=torch.float64,device='cuda'); f=torch.empty_like(sm); g=torch.empty_like(sm)
err=torch.zeros(S,dtype=torch.int32,device='cuda')
for name,fn in [('ssegrad',lambda: lib.sts_ewma_sse_gradient(x.data_ptr(),S,T,T,sm.data_ptr(),f.data_ptr(),g.data_ptr(),sp)),
                ('fit',lambda: lib.sts_ewma_fit(x.data_ptr(),S,T,T,sm.data_ptr(),err.data_ptr(),sp))]:
    fn(); torch.cuda.synchronize()
    t=time.perf_counter()
    for _ in range(3): fn()
    torch.cuda.synchronize(); print(name,(time.perf_counter()-t)/3*1e3,'ms',flush=True)
