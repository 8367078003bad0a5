"""ASP.NET Core Minimal-API conventions for the compat apps.

* responses: System.Text.Json web defaults — camelCase members (already the dict
  keys here), ``JavaScriptEncoder.Default`` escaping (non-ASCII and ``' " < > & +``
  as ``\\uXXXX``): :class:`NetJSONResponse`.
* request binding (``[FromBody]`` with web defaults): case-insensitive member names,
  numbers also accepted as JSON strings (``AllowReadingFromString``); a malformed
  body is a bare 400.
* ``Results.Problem`` -> ``application/problem+json``.
* optional ``UseHttpsRedirection`` (reference ``Program.cs:52``) as middleware.
"""
from __future__ import annotations

import json
from typing import Any, Optional

from starlette.responses import Response

from ..agent.dotnet_json import dumps as net_dumps
from ..agent.tools import Problem


class NetJSONResponse(Response):
    media_type = "application/json; charset=utf-8"

    def render(self, content: Any) -> bytes:
        return net_dumps(content).encode("utf-8")


def problem_response(p: Problem) -> Response:
    return Response(net_dumps(p.body).encode("utf-8"), status_code=p.status,
                    media_type="application/problem+json; charset=utf-8")


def respond(status: int, body: Any) -> Response:
    if isinstance(body, Problem):
        return problem_response(body)
    return NetJSONResponse(body, status_code=status)


class BindError(ValueError):
    pass


async def bind_body(request) -> dict:
    raw = await request.body()
    if not raw:
        raise BindError("Implicit body inferred for parameter but no body was provided.")
    try:
        val = json.loads(raw)
    except ValueError as e:
        raise BindError(str(e))
    if val is None:
        return {}
    if not isinstance(val, dict):
        raise BindError("body must be a JSON object")
    return val


def member(body: dict, name: str, kind: str = "string") -> Optional[Any]:
    """Case-insensitive member with web-default number handling."""
    val = None
    for k, v in body.items():
        if k.lower() == name.lower():
            val = v
    if val is None:
        return None
    if kind == "string":
        if not isinstance(val, str):
            raise BindError(f"The JSON value could not be converted to System.String. Path: $.{name}")
        return val
    if kind == "int":
        if isinstance(val, bool):
            raise BindError("invalid int")
        if isinstance(val, int):
            return val
        if isinstance(val, str) and val.strip().lstrip("-").isdigit():
            return int(val.strip())
        raise BindError(f"The JSON value could not be converted to System.Nullable`1[System.Int32]. Path: $.{name}")
    raise ValueError(kind)


def add_https_redirection(app, https_port: int):
    from starlette.middleware.base import BaseHTTPMiddleware
    from starlette.responses import RedirectResponse

    class _Redirect(BaseHTTPMiddleware):
        async def dispatch(self, request, call_next):
            if request.url.scheme == "http" and request.headers.get("x-forwarded-proto") != "https":
                url = request.url.replace(scheme="https", port=https_port)
                return RedirectResponse(str(url), status_code=307)
            return await call_next(request)

    app.add_middleware(_Redirect)
