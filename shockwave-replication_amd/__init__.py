"""MI355X-native Shockwave plan solver (drop-in for scheduler/shockwave.py).

The directory is also a flat module directory, like the reference's
``scheduler/``: put it on ``sys.path`` and ``from shockwave import
ShockwaveScheduler`` / ``from job_metadata import ShockwaveJobMetadata``
work exactly as in the reference.
"""
import os as _os
import sys as _sys

_HERE = _os.path.dirname(_os.path.abspath(__file__))
if _HERE not in _sys.path:
    _sys.path.insert(0, _HERE)

from job_metadata import ShockwaveJobMetadata  # noqa: E402,F401

__all__ = ["ShockwaveJobMetadata"]
