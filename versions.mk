# Single source of the release version and the toolchain versions the images use.
VERSION       ?= 0.1.0
ROCM_VERSION  ?= 7.2
IMAGE_NAME    ?= amdgpu-device-plugin
