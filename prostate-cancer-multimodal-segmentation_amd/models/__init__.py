"""Reference-shaped module path: pcms_amd.models.unet3d (models/unet3d.py)."""
