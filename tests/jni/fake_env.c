/* A fake JNI environment for tests/test_jni_glue.py: direct and heap
 * ByteBuffers, long[] / int[] / Object[] arrays and exception capture, so
 * capnp_packed_jni.c runs without a JVM.  Array elements are handed out as
 * copies (as a JVM may): Release with mode 0 copies back and frees, JNI_COMMIT
 * copies back, JNI_ABORT discards -- a missing or wrong release mode shows up
 * as unchanged output or a nonzero cpkt_outstanding(). */
#include <stdlib.h>
#include <string.h>

#include "jni.h"

enum { K_DIRECT = 1, K_HEAP, K_LONGS, K_INTS, K_OBJS, K_CLASS };
struct _jobject {
  int kind;
  void *addr;  /* buffer address / array data / jobject[] */
  int64_t cap; /* buffer capacity */
  jsize len;   /* array length */
  char name[96];
};

static char g_cls[96], g_msg[256];
static int g_pending, g_outstanding, g_local_refs;

static jclass FindClass(JNIEnv *env, const char *name) {
  (void)env;
  jclass c = (jclass)calloc(1, sizeof(struct _jobject));
  c->kind = K_CLASS;
  strncpy(c->name, name, sizeof c->name - 1);
  return c; /* (a local reference: leaked, as a test double may) */
}
static jint ThrowNew(JNIEnv *env, jclass c, const char *msg) {
  (void)env;
  if (g_pending) return -1; /* (the glue never throws twice) */
  g_pending = 1;
  strncpy(g_cls, c->name, sizeof g_cls - 1);
  strncpy(g_msg, msg ? msg : "", sizeof g_msg - 1);
  return 0;
}
static void DeleteLocalRef(JNIEnv *env, jobject o) {
  (void)env;
  (void)o;
  --g_local_refs;
}
static jsize GetArrayLength(JNIEnv *env, jarray a) {
  (void)env;
  return a->len;
}
static jobject GetObjectArrayElement(JNIEnv *env, jobjectArray a, jsize i) {
  (void)env;
  jobject o = ((jobject *)a->addr)[i];
  if (o) ++g_local_refs;
  return o;
}
static void *get_elems(jarray a, size_t es) {
  void *p = malloc((size_t)a->len * es + 1);
  memcpy(p, a->addr, (size_t)a->len * es);
  ++g_outstanding;
  return p;
}
static void release_elems(jarray a, void *p, jint mode, size_t es) {
  if (mode != JNI_ABORT) memcpy(a->addr, p, (size_t)a->len * es);
  if (mode != JNI_COMMIT) {
    free(p);
    --g_outstanding;
  }
}
static jlong *GetLongArrayElements(JNIEnv *env, jlongArray a, jboolean *c) {
  (void)env;
  if (c) *c = 1;
  return (jlong *)get_elems(a, 8);
}
static void ReleaseLongArrayElements(JNIEnv *env, jlongArray a, jlong *p, jint mode) {
  (void)env;
  release_elems(a, p, mode, 8);
}
static jint *GetIntArrayElements(JNIEnv *env, jintArray a, jboolean *c) {
  (void)env;
  if (c) *c = 1;
  return (jint *)get_elems(a, 4);
}
static void ReleaseIntArrayElements(JNIEnv *env, jintArray a, jint *p, jint mode) {
  (void)env;
  release_elems(a, p, mode, 4);
}
static void SetLongArrayRegion(JNIEnv *env, jlongArray a, jsize s, jsize n, const jlong *b) {
  (void)env;
  memcpy((jlong *)a->addr + s, b, (size_t)n * 8);
}
static void *GetDirectBufferAddress(JNIEnv *env, jobject b) {
  (void)env;
  return b && b->kind == K_DIRECT ? b->addr : NULL;
}
static jlong GetDirectBufferCapacity(JNIEnv *env, jobject b) {
  (void)env;
  return b && b->kind == K_DIRECT ? b->cap : -1;
}

static const struct JNINativeInterface_ g_table = {
    FindClass, ThrowNew, DeleteLocalRef, GetArrayLength, GetObjectArrayElement,
    GetLongArrayElements, ReleaseLongArrayElements, GetIntArrayElements, ReleaseIntArrayElements,
    SetLongArrayRegion, GetDirectBufferAddress, GetDirectBufferCapacity};
static JNIEnv g_env = &g_table;

JNIEnv *cpkt_env(void) { return &g_env; }
static jobject mk(int kind, void *addr, int64_t cap, jsize len) {
  jobject o = (jobject)calloc(1, sizeof(struct _jobject));
  o->kind = kind;
  o->addr = addr;
  o->cap = cap;
  o->len = len;
  return o;
}
jobject cpkt_direct(void *addr, int64_t cap) { return mk(K_DIRECT, addr, cap, 0); }
jobject cpkt_heap(int64_t cap) { return mk(K_HEAP, NULL, cap, 0); }
jobject cpkt_longs(int64_t *data, jsize len) { return mk(K_LONGS, data, 0, len); }
jobject cpkt_ints(int32_t *data, jsize len) { return mk(K_INTS, data, 0, len); }
jobject cpkt_objects(jobject *data, jsize len) { return mk(K_OBJS, data, 0, len); }
void cpkt_free(jobject o) { free(o); }
/* the pending exception (class, message): 1 if one was thrown */
int cpkt_exception(char *cls, char *msg) {
  strcpy(cls, g_cls);
  strcpy(msg, g_msg);
  return g_pending;
}
void cpkt_clear(void) {
  g_pending = 0;
  g_cls[0] = g_msg[0] = 0;
}
/* array elements not yet released + local references not deleted */
int cpkt_outstanding(void) { return g_outstanding + g_local_refs; }
