"""Reference-shaped module paths: pcms_amd.utils.losses / .trainer (utils/)."""
