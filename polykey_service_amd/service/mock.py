"""Mock tool backend with the reference's exact outputs (``internal/service/mock.go:14-67``).

* status is always ``{code: 200, message: "Tool executed successfully"}`` (``mock.go:24-29``)
* ``example_tool`` → string ``"Mock execution of example_tool at <RFC3339 now>"`` (``:33-36``)
* ``struct_tool``  → Struct ``{result:"success", timestamp:<unix>, data:{processed:true, count:42}}`` (``:37-51``)
* ``file_tool``    → File ``{example.txt, text/plain, "This is mock file content"}`` (``:52-59``)
* anything else    → string ``"Unknown tool: <name>"`` (``:60-63``)

``parameters``, ``secret_id`` and ``metadata`` are ignored, as in the reference.
"""
from __future__ import annotations

import datetime as _dt
import time
from typing import AsyncIterator, Optional

from .. import proto
from .base import RequestContext, ok_status

MOCK_TOOLS = ("example_tool", "struct_tool", "file_tool")


def rfc3339_now(now: Optional[_dt.datetime] = None) -> str:
    """Go ``time.Now().Format(time.RFC3339)``: second precision, ``Z`` or ``±hh:mm``."""
    now = now or _dt.datetime.now(_dt.timezone.utc).astimezone()
    off = now.utcoffset() or _dt.timedelta(0)
    if off == _dt.timedelta(0):
        return now.strftime("%Y-%m-%dT%H:%M:%SZ")
    mins = int(off.total_seconds() // 60)
    sign = "+" if mins >= 0 else "-"
    mins = abs(mins)
    return now.strftime("%Y-%m-%dT%H:%M:%S") + f"{sign}{mins // 60:02d}:{mins % 60:02d}"


def mock_response(tool_name: str) -> "proto.ExecuteToolResponse":
    resp = proto.ExecuteToolResponse(status=ok_status())
    if tool_name == "example_tool":
        resp.string_output = f"Mock execution of {tool_name} at {rfc3339_now()}"
    elif tool_name == "struct_tool":
        resp.struct_output.update({
            "result": "success",
            "timestamp": int(time.time()),
            "data": {"processed": True, "count": 42},
        })
    elif tool_name == "file_tool":
        resp.file_output.CopyFrom(proto.File(file_name="example.txt", mime_type="text/plain",
                                             content=b"This is mock file content"))
    else:
        resp.string_output = f"Unknown tool: {tool_name}"
    return resp


class MockService:
    """``service.NewMockService()`` equivalent."""

    async def execute_tool(self, ctx: RequestContext, tool_name: str, parameters=None,
                           secret_id: Optional[str] = None, metadata=None):
        return mock_response(tool_name)

    async def execute_tool_stream(self, ctx: RequestContext, tool_name: str, parameters=None,
                                  secret_id: Optional[str] = None, metadata=None) -> AsyncIterator:
        yield mock_response(tool_name)
