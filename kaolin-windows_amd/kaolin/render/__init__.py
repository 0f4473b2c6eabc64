from . import mesh  # noqa: F401
from . import spc  # noqa: F401
from . import camera  # noqa: F401
