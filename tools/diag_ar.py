import os, sys, numpy as np
sys.path.insert(0, "spark-timeseries_amd"); sys.path.insert(0, "oracle")
import torch, oracle
from sparkts import _native
from sparkts.models import Autoregression
_native.ensure_device(0)
S, T, p = 4300, 200, 3
x = oracle.gen_ar_panel(12, S, T, 3); x[17, T // 3] = np.nan
def run(lib, pers):
    _native._lib = _native.load_variant(lib)
    if pers: os.environ["STS_AR_PERS"] = "1"
    else: os.environ.pop("STS_AR_PERS", None)
    xd = torch.as_tensor(x, device="cuda:0")
    m, r = Autoregression.fitModelAndRemove(xd, p)
    m2 = Autoregression.fitModel(torch.as_tensor(x, device="cuda:0"), p)
    return m.c.cpu().numpy(), m.coefficients.cpu().numpy(), m2.c.cpu().numpy(), m2.coefficients.cpu().numpy()
_, rc, rcoef = oracle.panel_ar_fit_remove(x, p, threads=8)
for name, lib, pers in (("prod", _native.LIB_PATH if hasattr(_native, "LIB_PATH") else None, False), ("ab_pers", _native.AB_LIB_PATH, True), ("ab_nopers", _native.AB_LIB_PATH, False)):
    if lib is None: continue
    c, co, c2, co2 = run(lib, pers)
    d = np.nan_to_num(np.abs(c - c2)); dco = np.nan_to_num(np.abs(co - co2))
    bad = np.nonzero((d > 0) | (dco.max(1) > 0))[0]
    e = np.nanmax(np.abs(co - rcoef) / np.abs(rcoef)); e2 = np.nanmax(np.abs(co2 - rcoef) / np.abs(rcoef))
    print(name, "fused-vs-fitonly differing series:", len(bad), bad[:10], "max diff", d.max(), dco.max(), "rel vs oracle fused %.3g fitonly %.3g" % (e, e2))
