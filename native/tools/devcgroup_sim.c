/* libadp_devcgroup_sim.so: what a container's device cgroup does to the plugin,
 * without a container. LD_PRELOAD'ed into the daemon (or any amdsmi user), it
 * makes open()/openat() of /dev/kfd and /dev/dri/... fail with EPERM -- the
 * errno the devices controller returns for a character device the cgroup does
 * not allow (an unprivileged pod that only hostPath-mounts /dev). Everything
 * else, sysfs included, is untouched. ADP_DEVCGROUP_ALLOW="/dev/kfd" (colon
 * separated prefixes) re-allows nodes, to split the effect of each.
 * Test tooling only (tests/test_gpu.py::test_health_under_device_cgroup_denial).
 *
 * ADP_FS_WRITE_LOG=<file>: also append one line per filesystem write the process
 * attempts -- open/fopen for writing or creating, mkdir, rename, unlink, rmdir,
 * symlink, and bind() of a Unix socket -- "<call> <absolute path>", so a test
 * can check that every write lands on a volume the DaemonSet mounts (what a
 * read-only root filesystem requires). */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <sys/un.h>
#include <unistd.h>

/* The write log, written with raw syscalls (no recursion through the wrappers). */
static void log_write(const char* call, int dirfd, const char* path) {
  const char* log = getenv("ADP_FS_WRITE_LOG");
  if (!log || !path || !*path) return;
  char line[4352];
  char cwd[2048] = "";
  if (path[0] != '/') {
    if (dirfd != AT_FDCWD && dirfd >= 0) {
      char link[64];
      snprintf(link, sizeof(link), "/proc/self/fd/%d", dirfd);
      ssize_t n = readlink(link, cwd, sizeof(cwd) - 1);
      cwd[n > 0 ? n : 0] = 0;
    } else if (!getcwd(cwd, sizeof(cwd))) {
      cwd[0] = 0;
    }
  }
  int n = snprintf(line, sizeof(line), "%s %s%s%s\n", call, cwd, cwd[0] ? "/" : "", path);
  if (n <= 0) return;
  if (n >= (int)sizeof(line)) n = (int)sizeof(line) - 1;
  int fd = (int)syscall(SYS_openat, AT_FDCWD, log, O_WRONLY | O_APPEND | O_CREAT | O_CLOEXEC, 0644);
  if (fd < 0) return;
  ssize_t w = syscall(SYS_write, fd, line, (size_t)n);
  (void)w;
  syscall(SYS_close, fd);
}

/* (__O_TMPFILE includes O_DIRECTORY's bit: an opendir() is no write) */
static int writes(int flags) {
  return (flags & (O_WRONLY | O_RDWR | O_CREAT | O_TRUNC)) != 0 || (flags & __O_TMPFILE) == __O_TMPFILE;
}

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
    if (writes(flags)) log_write(#name, AT_FDCWD, path);                    \
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
    if (writes(flags)) log_write(#name, dirfd, path);                       \
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
static int mode_writes(const char* mode) { return mode && strpbrk(mode, "wa+") != NULL; }

FILE* fopen(const char* path, const char* mode) {
  if (denied(path)) { errno = EPERM; return NULL; }
  if (mode_writes(mode)) log_write("fopen", AT_FDCWD, path);
  static FILE* (*real)(const char*, const char*);
  if (!real) real = (FILE * (*)(const char*, const char*)) dlsym(RTLD_NEXT, "fopen");
  return real(path, mode);
}
FILE* fopen64(const char* path, const char* mode) {
  if (denied(path)) { errno = EPERM; return NULL; }
  if (mode_writes(mode)) log_write("fopen64", AT_FDCWD, path);
  static FILE* (*real)(const char*, const char*);
  if (!real) real = (FILE * (*)(const char*, const char*)) dlsym(RTLD_NEXT, "fopen64");
  return real(path, mode);
}

/* The other writes, logged only (ADP_FS_WRITE_LOG) and passed through. */
#define REAL(ret, name, ...) \
  static ret (*real)(__VA_ARGS__); \
  if (!real) real = (ret (*)(__VA_ARGS__))dlsym(RTLD_NEXT, #name)

int mkdir(const char* path, mode_t m) {
  REAL(int, mkdir, const char*, mode_t);
  log_write("mkdir", AT_FDCWD, path);
  return real(path, m);
}
int mkdirat(int d, const char* path, mode_t m) {
  REAL(int, mkdirat, int, const char*, mode_t);
  log_write("mkdirat", d, path);
  return real(d, path, m);
}
int rename(const char* a, const char* b) {
  REAL(int, rename, const char*, const char*);
  log_write("rename", AT_FDCWD, b);
  return real(a, b);
}
int renameat(int da, const char* a, int db, const char* b) {
  REAL(int, renameat, int, const char*, int, const char*);
  log_write("renameat", db, b);
  return real(da, a, db, b);
}
int unlink(const char* path) {
  REAL(int, unlink, const char*);
  log_write("unlink", AT_FDCWD, path);
  return real(path);
}
int unlinkat(int d, const char* path, int flags) {
  REAL(int, unlinkat, int, const char*, int);
  log_write("unlinkat", d, path);
  return real(d, path, flags);
}
int rmdir(const char* path) {
  REAL(int, rmdir, const char*);
  log_write("rmdir", AT_FDCWD, path);
  return real(path);
}
int symlink(const char* target, const char* path) {
  REAL(int, symlink, const char*, const char*);
  log_write("symlink", AT_FDCWD, path);
  return real(target, path);
}
int bind(int fd, const struct sockaddr* addr, socklen_t len) {
  REAL(int, bind, int, const struct sockaddr*, socklen_t);
  if (addr && addr->sa_family == AF_UNIX && len > sizeof(sa_family_t)) {
    const struct sockaddr_un* un = (const struct sockaddr_un*)addr;
    if (un->sun_path[0]) log_write("bind", AT_FDCWD, un->sun_path);  /* abstract sockets write nothing */
  }
  return real(fd, addr, len);
}
