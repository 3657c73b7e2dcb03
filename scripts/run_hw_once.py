"""One HW-DFMI + one ortho fit (3 buffers, 1 record) for counter collection."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from deepfmkit_amd import fitters as F  # noqa: E402

G = np.load(os.path.join(ROOT, "tests", "golden", "wdfmi.npz"))
f_samp, f_mod, df, meas, ref, f_ref, n = G["cos_cfg"]
R = 4000
main = G["cos_main"][: 3 * R]
tau0 = (meas - ref) / 299792458.0
for _ in range(2):
    F.wdfmi_records("hwdfmi", main[None], G["cos_hw_witness"], f_samp, f_mod, R, 3, df=df, tau_init=tau0, f_ref=f_ref)
    F.wdfmi_records("wdfmi_ortho", main[None], G["cos_witness"], f_samp, f_mod, R, 3, df=df, tau_init=tau0, init_psi=0.3)
print("ok")
