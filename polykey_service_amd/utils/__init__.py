from . import slog

__all__ = ["slog"]
