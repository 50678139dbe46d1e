"""MCP tool server (JSON-RPC 2.0 over stdio / streamable HTTP) and the HTTP
bridge (:3333) -- reference: fastmcp/server.py, mcp/src/index.ts."""
