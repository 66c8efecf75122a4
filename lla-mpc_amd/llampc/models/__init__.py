from llampc.models.model import Model  # noqa: F401
from llampc.models.dynamic import Dynamic  # noqa: F401
