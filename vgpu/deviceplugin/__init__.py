"""vgpu.deviceplugin."""
