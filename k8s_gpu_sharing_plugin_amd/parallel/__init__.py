"""See package docstring in k8s_gpu_sharing_plugin_amd/__init__.py."""
