/*
 * A stand-in libhdfs.so for tests: the libhdfs C API (hdfs.h) over a local
 * directory ($FAKE_HDFS_ROOT), so the hdfs:// backend's dlopen path, symbol
 * table, stream loop and listing run end to end without a JVM or a cluster.
 * "hdfs://host:port/a/b" maps to $FAKE_HDFS_ROOT/a/b; listings return full
 * hdfs:// URIs the way the real library does.  Reads are capped at 1000 bytes
 * and fail once with EINTR, exercising the backend's short-read/retry loop.
 */
#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

typedef int32_t tSize;
typedef int64_t tOffset;
typedef int64_t tTime;
typedef enum { kObjectKindFile = 'F', kObjectKindDirectory = 'D' } tObjectKind;
typedef struct {
  tObjectKind mKind;
  char* mName;
  tTime mLastMod;
  tOffset mSize;
  short mReplication;
  tOffset mBlockSize;
  char* mOwner;
  char* mGroup;
  short mPermissions;
  tTime mLastAccess;
} hdfsFileInfo;

typedef struct {
  char prefix[256]; /* "hdfs://host:port" */
} FakeFS;

typedef struct {
  int fd;
} FakeFile;

static int g_eintr_once = 1;

static void local_path(const char* uri, char* out, size_t n) {
  const char* root = getenv("FAKE_HDFS_ROOT");
  const char* p = strstr(uri, "://");
  if (p != NULL) {
    p = strchr(p + 3, '/');
    if (p == NULL) p = "/";
  } else {
    p = uri;
  }
  snprintf(out, n, "%s%s", root ? root : "", p);
}

void* hdfsConnect(const char* host, uint16_t port) {
  FakeFS* fs = (FakeFS*)calloc(1, sizeof(FakeFS));
  snprintf(fs->prefix, sizeof(fs->prefix), "hdfs://%s:%u", host, (unsigned)port);
  return fs;
}

int hdfsDisconnect(void* fs) {
  free(fs);
  return 0;
}

void* hdfsOpenFile(void* fs, const char* path, int flags, int bufsize, short rep, tSize block) {
  (void)fs;
  (void)bufsize;
  (void)rep;
  (void)block;
  char lp[4096];
  local_path(path, lp, sizeof(lp));
  if (flags & O_WRONLY) { /* HDFS creates missing parent directories */
    for (char* q = strchr(lp + 1, '/'); q != NULL; q = strchr(q + 1, '/')) {
      *q = '\0';
      mkdir(lp, 0755);
      *q = '/';
    }
  }
  int f = (flags & O_WRONLY) ? (flags | O_CREAT | ((flags & O_APPEND) ? 0 : O_TRUNC)) : O_RDONLY;
  int fd = open(lp, f, 0644);
  if (fd < 0) return NULL;
  FakeFile* h = (FakeFile*)calloc(1, sizeof(FakeFile));
  h->fd = fd;
  return h;
}

int hdfsCloseFile(void* fs, void* file) {
  (void)fs;
  FakeFile* h = (FakeFile*)file;
  close(h->fd);
  free(h);
  return 0;
}

tSize hdfsRead(void* fs, void* file, void* buf, tSize len) {
  (void)fs;
  if (g_eintr_once) {
    g_eintr_once = 0;
    errno = EINTR;
    return -1;
  }
  if (len > 1000) len = 1000;
  return (tSize)read(((FakeFile*)file)->fd, buf, (size_t)len);
}

tSize hdfsWrite(void* fs, void* file, const void* buf, tSize len) {
  (void)fs;
  if (len > 4096) len = 4096; /* short writes: the caller must loop */
  return (tSize)write(((FakeFile*)file)->fd, buf, (size_t)len);
}

int hdfsSeek(void* fs, void* file, tOffset pos) {
  (void)fs;
  return lseek(((FakeFile*)file)->fd, pos, SEEK_SET) < 0 ? -1 : 0;
}

tOffset hdfsTell(void* fs, void* file) {
  (void)fs;
  return lseek(((FakeFile*)file)->fd, 0, SEEK_CUR);
}

int hdfsFlush(void* fs, void* file) {
  (void)fs;
  (void)file;
  return 0;
}

static void fill_info(hdfsFileInfo* fi, const char* name, const struct stat* st) {
  memset(fi, 0, sizeof(*fi));
  fi->mKind = S_ISDIR(st->st_mode) ? kObjectKindDirectory : kObjectKindFile;
  fi->mName = strdup(name);
  fi->mSize = S_ISDIR(st->st_mode) ? 0 : st->st_size;
  fi->mReplication = 3;
  fi->mBlockSize = 128 << 20;
}

hdfsFileInfo* hdfsGetPathInfo(void* fs, const char* path) {
  (void)fs;
  char lp[4096];
  struct stat st;
  local_path(path, lp, sizeof(lp));
  if (stat(lp, &st) != 0) return NULL;
  hdfsFileInfo* fi = (hdfsFileInfo*)malloc(sizeof(hdfsFileInfo));
  fill_info(fi, path, &st);
  return fi;
}

static int by_name(const void* a, const void* b) {
  return strcmp(*(char* const*)a, *(char* const*)b);
}

hdfsFileInfo* hdfsListDirectory(void* fs, const char* path, int* n) {
  FakeFS* f = (FakeFS*)fs;
  char lp[4096];
  local_path(path, lp, sizeof(lp));
  *n = 0;
  DIR* d = opendir(lp);
  if (d == NULL) return NULL;
  hdfsFileInfo* out = (hdfsFileInfo*)calloc(256, sizeof(hdfsFileInfo));
  char* names[256];
  int k = 0;
  struct dirent* e;
  while ((e = readdir(d)) != NULL && k < 256) {
    if (e->d_name[0] != '.') names[k++] = strdup(e->d_name);
  }
  closedir(d);
  qsort(names, (size_t)k, sizeof(char*), by_name);  /* the namenode lists in name order */
  const char* rel = strstr(path, "://") ? strchr(strstr(path, "://") + 3, '/') : path;
  for (int i = 0; i < k; ++i) {
    char full[8192], name[8192];
    struct stat st;
    snprintf(full, sizeof(full), "%s/%s", lp, names[i]);
    if (stat(full, &st) == 0) {
      snprintf(name, sizeof(name), "%s%s/%s", f->prefix, rel ? rel : "", names[i]);
      fill_info(&out[(*n)++], name, &st);
    }
    free(names[i]);
  }
  return out;
}

void hdfsFreeFileInfo(hdfsFileInfo* info, int n) {
  for (int i = 0; i < n; ++i) free(info[i].mName);
  free(info);
}
