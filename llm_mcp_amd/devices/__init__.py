"""GPU fleet: ROCm device enumeration and the discovery runner."""
