from .jest import print_jest_report
from .log_beautifier import Beautifier

__all__ = ["print_jest_report", "Beautifier"]
