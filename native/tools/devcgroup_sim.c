/* libadp_devcgroup_sim.so: what a container's device cgroup does to the plugin,
 * without a container. LD_PRELOAD'ed into the daemon (or any amdsmi user), it
 * makes open()/openat() of /dev/kfd and /dev/dri/... fail with EPERM -- the
 * errno the devices controller returns for a character device the cgroup does
 * not allow (an unprivileged pod that only hostPath-mounts /dev). Everything
 * else, sysfs included, is untouched. ADP_DEVCGROUP_ALLOW="/dev/kfd" (colon
 * separated prefixes) re-allows nodes, to split the effect of each.
 * Test tooling only (tests/test_gpu.py::test_health_under_device_cgroup_denial). */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int denied(const char* path) {
  if (!path) return 0;
  if (strcmp(path, "/dev/kfd") != 0 && strncmp(path, "/dev/dri/", 9) != 0) return 0;
  const char* allow = getenv("ADP_DEVCGROUP_ALLOW");
  while (allow && *allow) {
    const char* end = strchr(allow, ':');
    size_t n = end ? (size_t)(end - allow) : strlen(allow);
    if (n && strncmp(path, allow, n) == 0) return 0;
    allow = end ? end + 1 : NULL;
  }
  if (getenv("ADP_DEVCGROUP_VERBOSE")) fprintf(stderr, "devcgroup_sim: open(%s) -> EPERM\n", path);
  return 1;
}

static mode_t mode_arg(int flags, va_list ap) {
  return (flags & (O_CREAT | __O_TMPFILE)) ? (mode_t)va_arg(ap, int) : 0;
}

#define WRAP_OPEN(name)                                                     \
  int name(const char* path, int flags, ...) {                             \
    va_list ap;                                                             \
    va_start(ap, flags);                                                    \
    mode_t m = mode_arg(flags, ap);                                         \
    va_end(ap);                                                             \
    if (denied(path)) { errno = EPERM; return -1; }                         \
    static int (*real)(const char*, int, ...);                              \
    if (!real) real = (int (*)(const char*, int, ...))dlsym(RTLD_NEXT, #name); \
    return real(path, flags, m);                                            \
  }
WRAP_OPEN(open)
WRAP_OPEN(open64)

#define WRAP_OPENAT(name)                                                   \
  int name(int dirfd, const char* path, int flags, ...) {                  \
    va_list ap;                                                             \
    va_start(ap, flags);                                                    \
    mode_t m = mode_arg(flags, ap);                                         \
    va_end(ap);                                                             \
    if (denied(path)) { errno = EPERM; return -1; }                         \
    static int (*real)(int, const char*, int, ...);                         \
    if (!real) real = (int (*)(int, const char*, int, ...))dlsym(RTLD_NEXT, #name); \
    return real(dirfd, path, flags, m);                                     \
  }
WRAP_OPENAT(openat)
WRAP_OPENAT(openat64)

/* _FORTIFY_SOURCE variants */
int __open_2(const char* path, int flags) { return open(path, flags); }
int __open64_2(const char* path, int flags) { return open64(path, flags); }
int __openat_2(int d, const char* path, int flags) { return openat(d, path, flags); }
int __openat64_2(int d, const char* path, int flags) { return openat64(d, path, flags); }

/* fopen() opens through an internal, non-interposable open: wrap it too. */
FILE* fopen(const char* path, const char* mode) {
  if (denied(path)) { errno = EPERM; return NULL; }
  static FILE* (*real)(const char*, const char*);
  if (!real) real = (FILE * (*)(const char*, const char*)) dlsym(RTLD_NEXT, "fopen");
  return real(path, mode);
}
FILE* fopen64(const char* path, const char* mode) {
  if (denied(path)) { errno = EPERM; return NULL; }
  static FILE* (*real)(const char*, const char*);
  if (!real) real = (FILE * (*)(const char*, const char*)) dlsym(RTLD_NEXT, "fopen64");
  return real(path, mode);
}
