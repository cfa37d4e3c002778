"""``python -m polykey_service_amd.report [jest|beautify]`` (default: beautify, a stdin filter)."""
import sys

from . import jest, log_beautifier

mode = sys.argv[1] if len(sys.argv) > 1 else "beautify"
sys.exit(jest.main() if mode == "jest" else log_beautifier.main())
