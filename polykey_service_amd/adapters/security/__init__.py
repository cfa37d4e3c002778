from . import cipher
from .secret_store import SecretStore, parse_key

__all__ = ["cipher", "SecretStore", "parse_key"]
