"""A Molly-format producer: Dedalus evaluation with provenance, lineage-driven
fault injection and the output files faultinjectors/molly.go reads (SURVEY.md
§8f row 1).  Input generator for the case-study configurations; not part of the
device path."""
from .dedalus import FailureSpec, Program, Run, evaluate, parse  # noqa: F401
from .ldfi import explore, write_output  # noqa: F401
