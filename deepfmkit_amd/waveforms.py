"""Modulation waveforms of the reference (waveforms.py) for LaserConfig.waveform_func.

They feed the asd-mode generator (physics.exact_model_signal, reference
physics.py:615-722) on the host; the device trial generator (dfmi_synth_asd) covers
`cosine_waveform` and `second_harmonic_distortion` (synth.h).

Reference map: second_harmonic_distortion waveforms.py:4-23, triangle_wave :25-31,
square_wave :33-43, dfm_like_wave :45-65, dfm_wave :67-90.
"""
from __future__ import annotations

import numpy as np

from .physics import cosine_waveform  # noqa: F401  (the default waveform)


def second_harmonic_distortion(t_phase, distortion_amp=0.0, distortion_phase=0.0):
    """cos(t) + distortion_amp * cos(2 t + distortion_phase), numpy's operation order."""
    fundamental = np.cos(t_phase)
    second_harmonic = distortion_amp * np.cos(2 * t_phase + distortion_phase)
    return fundamental + second_harmonic


def triangle_wave(t_phase, width=0.5):
    """scipy.signal.sawtooth with width 0.5 (a triangle)."""
    from scipy.signal import sawtooth
    return sawtooth(t_phase, width=width)


def square_wave(t_phase, duty=0.5):
    """scipy.signal.square with the given duty cycle."""
    from scipy.signal import square
    return square(t_phase, duty=duty)


def dfm_like_wave(t_phase, harmonics=None):
    """cos(t) + sum_n a_n cos(n t) (default {2: 0.1, 3: 0.05})."""
    if harmonics is None:
        harmonics = {2: 0.1, 3: 0.05}
    y = np.cos(t_phase)
    for n, amp in harmonics.items():
        y += amp * np.cos(n * t_phase)
    return y


def dfm_wave(t_phase, m=1.0, phi=0.0):
    """cos(phi + m cos(t)): the AC shape of an inner DFMI signal."""
    return np.cos(phi + m * np.cos(t_phase))
