from pysnptools_amd.standardizer.standardizer import Standardizer
from pysnptools_amd.standardizer.beta import Beta
from pysnptools_amd.standardizer.unit import Unit
from pysnptools_amd.standardizer.identity import Identity
from pysnptools_amd.standardizer.diag_K_to_N import DiagKtoN, DiagKtoNTrained
from pysnptools_amd.standardizer.betatrained import BetaTrained
from pysnptools_amd.standardizer.unittrained import UnitTrained
