"""`python -m pconv image.raw W H reps {grey,rgb} [options]` — the reference CLI."""
import sys

from .utils.cli import main

sys.exit(main(sys.argv))
