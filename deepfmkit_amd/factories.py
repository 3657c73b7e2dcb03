"""Experiment configuration factories (reference factories.py).

An ExperimentFactory turns one trial's parameter dict into the physics objects of
that trial ({'laser_config', 'main_ifo_config'[, 'witness_ifo_config']}); the
Experiment runner (experiments.py) calls it once per trial, in the parent process.

Reference map: ExperimentFactory factories.py:7-44, StandardDFMIExperimentFactory
:47-110, StandardWDFMIExperimentFactory :112-180, VairableAmplitudeOffset :186-221
(the reference's spelling, kept for drop-in use).
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Callable, Set

import numpy as np
import scipy.constants as sc

from . import physics


class ExperimentFactory(ABC):
    """factories.py:7-44."""

    @abstractmethod
    def __call__(self, params: dict) -> dict:
        ...

    @abstractmethod
    def _get_expected_params_keys(self) -> Set[str]:
        ...


class StandardDFMIExperimentFactory(ExperimentFactory):
    """factories.py:47-110: one main interferometer of OPD `opd_main`, m_main sets df."""

    def __init__(self, waveform_function: Callable, opd_main: float = 0.1):
        if not callable(waveform_function):
            raise TypeError("waveform_function must be a callable.")
        self.waveform_func_to_use = waveform_function
        self.opd_main = opd_main

    def _get_expected_params_keys(self) -> Set[str]:
        return {"m_main", "psi", "phi", "distortion_amp", "distortion_phase", "waveform_kwargs"}

    def __call__(self, params: dict) -> dict:
        m_main = params["m_main"]
        waveform_kwargs = {"distortion_amp": params.get("distortion_amp", 0.0),
                           "distortion_phase": params.get("distortion_phase", 0.0)}
        laser = physics.LaserConfig()
        laser.psi = params.get("psi", 0)
        ifo = physics.InterferometerConfig(label="main_ifo")
        ifo.ref_arml = 0.1
        ifo.meas_arml = ifo.ref_arml + self.opd_main
        ifo.phi = params.get("phi", 0)
        laser.waveform_func = self.waveform_func_to_use
        laser.waveform_kwargs = waveform_kwargs
        laser.df = (m_main * sc.c) / (2 * np.pi * self.opd_main)
        return {"laser_config": laser, "main_ifo_config": ifo}


class StandardWDFMIExperimentFactory(ExperimentFactory):
    """factories.py:112-180: main interferometer + a static witness of modulation depth
    m_witness sharing the laser."""

    def __init__(self, waveform_function: Callable, opd_main: float = 0.2):
        if not callable(waveform_function):
            raise TypeError("waveform_function must be a callable.")
        self.waveform_func_to_use = waveform_function
        self.opd_main = opd_main

    def _get_expected_params_keys(self) -> Set[str]:
        return {"m_main", "m_witness", "psi", "phi", "distortion_amp", "distortion_phase", "waveform_kwargs"}

    def __call__(self, params: dict) -> dict:
        m_main = params["m_main"]
        m_witness = params.get("m_witness", 0.0)
        waveform_kwargs = {"distortion_amp": params.get("distortion_amp", 0.0),
                           "distortion_phase": params.get("distortion_phase", 0.0)}
        laser = physics.LaserConfig()
        laser.psi = params.get("psi", 0)
        ifo = physics.InterferometerConfig(label="main_ifo")
        ifo.ref_arml = 0.1
        ifo.meas_arml = ifo.ref_arml + self.opd_main
        ifo.phi = params.get("phi", 0)
        laser.waveform_func = self.waveform_func_to_use
        laser.waveform_kwargs = waveform_kwargs
        laser.df = (m_main * sc.c) / (2 * np.pi * self.opd_main)
        wit = physics.InterferometerConfig(label="witness_ifo")
        if laser.df > 0 and m_witness > 0:
            opd_witness = (m_witness * sc.c) / (2 * np.pi * laser.df)
            wit.ref_arml = 0.01
            wit.meas_arml = wit.ref_arml + opd_witness
            f0 = sc.c / laser.wavelength
            static_fringe_phase = (2 * np.pi * f0 * opd_witness) / sc.c
            wit.phi = (np.pi / 2.0) - static_fringe_phase
        return {"laser_config": laser, "main_ifo_config": ifo, "witness_ifo_config": wit}


class VairableAmplitudeOffset(ExperimentFactory):
    """factories.py:186-221: laser amplitude = nominal_amplitude + amplitude_offset
    (notebooks/5.0_Experiment)."""

    def __init__(self, opd_main: float = 0.1):
        self.opd_main = opd_main

    def _get_expected_params_keys(self) -> Set[str]:
        return {"m_main", "nominal_amplitude", "amplitude_offset", "waveform_kwargs"}

    def __call__(self, params: dict) -> dict:
        laser = physics.LaserConfig(label="ExperimentLaser")
        laser.amp = params["nominal_amplitude"] + params["amplitude_offset"]
        if self.opd_main == 0:
            raise ValueError("opd_main cannot be zero in the factory.")
        laser.df = (params["m_main"] * sc.c) / (2 * np.pi * self.opd_main)
        ifo = physics.InterferometerConfig(label="main_ifo")
        ifo.ref_arml = 0.1
        ifo.meas_arml = ifo.ref_arml + self.opd_main
        return {"laser_config": laser, "main_ifo_config": ifo}
