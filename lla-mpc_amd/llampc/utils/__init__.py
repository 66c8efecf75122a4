from llampc.utils.spline import Spline, Spline2D  # noqa: F401
from llampc.utils.projection import Projection, project_segments  # noqa: F401
