'''
MI355X dense simplex pivot engine behind the lpsol Tableau/Simplex API
(reference: tkoz0/linear-program-solver, lpsol/__init__.py:5-17).
'''

from .tableau import Tableau
from .simplex import Simplex
from .linprog import LinProg
from ._lib import Engine, EngineUnavailable, DeviceError

__all__ = [
    'Tableau',
    'Simplex',
    'LinProg',
    'Engine',
    'EngineUnavailable',
    'DeviceError',
]
