"""Import alias: makes the package directory `indoor-nerf_amd/` importable as `indoor_nerf_amd`
(a hyphen is not a valid Python identifier). This module acts as the package's __init__: it sets
__path__ to that directory and re-exports its public API."""
import os as _os

__path__ = [_os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "indoor-nerf_amd")]

from indoor_nerf_amd.api import *  # noqa: E402,F401,F403
from indoor_nerf_amd.api import __all__  # noqa: E402,F401
