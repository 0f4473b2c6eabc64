from . import mesh  # noqa: F401
from . import conversions  # noqa: F401
from . import spc  # noqa: F401
from . import pointcloud  # noqa: F401
