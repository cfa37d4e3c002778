from .base import RequestContext, Service, ToolError, ok_status
from .mock import MOCK_TOOLS, MockService, mock_response, rfc3339_now
from .router import ToolRouter, make_default_router

__all__ = ["RequestContext", "Service", "ToolError", "ok_status", "MOCK_TOOLS", "MockService",
           "mock_response", "rfc3339_now", "ToolRouter", "make_default_router"]
