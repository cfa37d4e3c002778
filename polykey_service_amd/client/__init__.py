from .dev_client import CHANNEL_OPTIONS, Client, build_request, create_connection, main, run, wait_for_connection

__all__ = ["CHANNEL_OPTIONS", "Client", "build_request", "create_connection", "main", "run", "wait_for_connection"]
