"""Test-only stand-in for the PyDP package (python-dp==1.1.3rc2), which is
not installed in this container.

CONTAINER-ONLY TEST INFRASTRUCTURE: used solely by oracle/gen_golden.py to
import the reference pipeline_dp for noise-free golden vectors.  Noise is the
identity and partition selection keeps everything, so the reference's
LocalBackend becomes a deterministic (modulo numpy sampling) oracle for the
bounding / accumulation / formula path.  Never imported by product code and
never shipped to or used on the GPU box.
"""
from . import algorithms  # noqa: F401
from . import _pydp  # noqa: F401
