#!/bin/sh
# Copy the enforcement library to the host dir Allocate mounts into containers
# (reference docker/entrypoint.sh:17-21), then run the requested component.
set -e
if [ -d /usr/local/vgpu ]; then
  cp -f /opt/vgpu/vgpu/_lib/libvgpu.so /usr/local/vgpu/libvgpu.so.new && mv -f /usr/local/vgpu/libvgpu.so.new /usr/local/vgpu/libvgpu.so
  echo /usr/local/vgpu/libvgpu.so > /usr/local/vgpu/ld.so.preload
fi
exec "$@"
