"""deepfmkit_amd — MI355X-native DFMI per-segment NLS readout engine.

Drop-in for the hot path of mdovale/DeepFMKit: `DeepFitFramework.fit()` with the
'nls' and 'ekf' strategies, the fit.* module constants, and the workers entry
points. All arithmetic of the path runs in hand-written HIP kernels for gfx950
(libdfmi.so, C ABI in include/dfmi.h); there is no CPU fallback.
"""
from . import fit  # noqa: F401
from .core import DeepFitFramework, vectorized_downsample  # noqa: F401
from .data import DeepFitObject, DeepRawObject  # noqa: F401
from .fitters import BaseFitter, EKFFitter, StandardNLSFitter  # noqa: F401
from .physics import (DFMIObject, InterferometerConfig, LaserConfig, SignalGenerator,  # noqa: F401
                      set_laser_df_for_effect)

__version__ = "0.1.0"
