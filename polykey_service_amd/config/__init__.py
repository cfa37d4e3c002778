from .goflag import FlagError, FlagSet
from .loader import Config, ConfigLoader, NetworkTester, split_host_port
from .runtime import RuntimeDetector, RuntimeEnvironment
from .server_config import ServerConfig, load_server_config

__all__ = ["FlagError", "FlagSet", "Config", "ConfigLoader", "NetworkTester", "split_host_port",
           "RuntimeDetector", "RuntimeEnvironment", "ServerConfig", "load_server_config"]
