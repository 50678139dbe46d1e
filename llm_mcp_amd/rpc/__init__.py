"""llmmcp.v1.Core gRPC contract: runtime-built protobuf classes (no protoc /
grpc_tools in this image), server over the store, and a client."""
