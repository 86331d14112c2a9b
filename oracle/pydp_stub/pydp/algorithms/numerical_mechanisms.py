"""Test-only stub of pydp.algorithms.numerical_mechanisms: identity noise.

The std / diversity values use the oracle's restatement of PyDP's calibration
so explain-computation strings and std helpers stay meaningful.
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", ".."))
from pdp_oracle import gaussian_sigma  # noqa: E402


class LaplaceMechanism:

    def __init__(self, epsilon, sensitivity):
        self.epsilon = epsilon
        self.sensitivity = sensitivity
        self.diversity = sensitivity / epsilon

    def add_noise(self, value):
        return value


class GaussianMechanism:

    def __init__(self, epsilon, delta, l2_sensitivity):
        self.epsilon = epsilon
        self.delta = delta
        self.l2_sensitivity = l2_sensitivity
        self.std = gaussian_sigma(epsilon, delta, l2_sensitivity)

    def add_noise(self, value):
        return value
