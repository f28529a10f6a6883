# Convenience targets (reference Makefile:1-33 builds the Go binaries).
PY ?= python3

.PHONY: all native kernels test test-gpu bench suite vmem clean chart-lint

all: native

native:
	$(PY) -m vgpu.native.build all

kernels:
	$(PY) -m vgpu.native.build kernels

test:
	$(PY) -m pytest tests -m "not gpu" -q

test-gpu:
	$(PY) -m pytest tests -m gpu -q

bench:
	$(PY) bench.py

suite:
	$(PY) -m vgpu.bench.suite

vmem:
	$(PY) -m vgpu.bench.vmem

clean:
	$(PY) -m vgpu.native.build clean
