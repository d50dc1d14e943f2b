"""pyrr stand-in (FIXTURE-GENERATION ONLY): only matrix44.create_look_at."""
from . import matrix44  # noqa: F401
