/*
 * capnp_packed_jni.c -- JNI glue between org.capnproto.gpu.PackedGpu and the
 * C ABI of include/capnp_packed.h.  Built where a JDK exists (this image has
 * none; INTEGRATION.md gives the command):
 *
 *   cc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux \
 *      -I../../../include capnp_packed_jni.c \
 *      -L../../lib -lcapnp_packed_hip -Wl,-rpath,'$ORIGIN' -o libcapnp_packed_jni.so
 *
 * Buffers: every ByteBuffer argument must be direct and is passed zero-copy
 * (GetDirectBufferAddress; DIRECT allocation exists in the reference,
 * DefaultAllocator.java:56-62); a heap buffer is rejected with CPK_EINVAL --
 * PackedGpu.java copies heap buffers into direct ones before calling in.
 * Array lengths, positions and buffer capacities are checked here before the
 * library sees a pointer.  Status
 * codes become the reference's exceptions: decode errors ->
 * org.capnproto.DecodeException (DecodeException.java:24-27), device / memory
 * errors -> java.io.IOException.
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "capnp_packed.h"

static void throw_status(JNIEnv *env, int st) {
  const char *cls = (st == CPK_ETRUNC || st == CPK_EOVERRUN || st == CPK_ETRAILING ||
                     st == CPK_EINVAL || st == CPK_EFRAME)
                        ? "org/capnproto/DecodeException"
                        : "java/io/IOException";
  /* (the message is cpk_status_string's: PackedGpu.TRUNCATED tells a
     truncation apart, DecodeException being final) */
  jclass c = (*env)->FindClass(env, cls);
  if (c) (*env)->ThrowNew(env, c, cpk_status_string(st));
}

/* an offset array of n + 1 entries needs length >= 1 */
static int offsets_ok(JNIEnv *env, jlongArray a) { return a && (*env)->GetArrayLength(env, a) >= 1; }

/* piece i of a gather: buffer b from pos for `bytes` bytes, inside its capacity */
static const void *gather_ptr(JNIEnv *env, jobject b, jint pos, uint64_t bytes, int *st) {
  uint8_t *a = b ? (uint8_t *)(*env)->GetDirectBufferAddress(env, b) : NULL;
  jlong cap = b ? (*env)->GetDirectBufferCapacity(env, b) : -1;
  if (bytes == 0) return a ? a + (pos > 0 ? pos : 0) : NULL;  /* (an empty piece needs no buffer) */
  if (!a || pos < 0 || cap < 0 || (uint64_t)cap < (uint64_t)pos || (uint64_t)cap - (uint64_t)pos < bytes) {
    *st = CPK_EINVAL;
    return NULL;
  }
  return a + pos;
}

/* long PackedGpu.nativeCreate(int device) */
JNIEXPORT jlong JNICALL Java_org_capnproto_gpu_PackedGpu_nativeCreate(JNIEnv *env, jclass k,
                                                                       jint device) {
  (void)k;
  cpk_ctx ctx = NULL;
  int st = cpk_ctx_create(device, &ctx);
  if (st != CPK_OK) {
    throw_status(env, st);
    return 0;
  }
  return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JNICALL Java_org_capnproto_gpu_PackedGpu_nativeDestroy(JNIEnv *env, jclass k,
                                                                      jlong h) {
  (void)env;
  (void)k;
  cpk_ctx_destroy((cpk_ctx)(intptr_t)h);
}

JNIEXPORT jlong JNICALL Java_org_capnproto_gpu_PackedGpu_nativeCapacity(JNIEnv *env, jclass k,
                                                                        jlongArray segWordOff) {
  (void)k;
  if (!offsets_ok(env, segWordOff)) {
    throw_status(env, CPK_EINVAL);
    return 0;
  }
  jsize n1 = (*env)->GetArrayLength(env, segWordOff);
  jlong *swo = (*env)->GetLongArrayElements(env, segWordOff, NULL);
  uint64_t cap = cpk_batch_packed_capacity((const uint64_t *)swo, (uint32_t)(n1 - 1));
  (*env)->ReleaseLongArrayElements(env, segWordOff, swo, JNI_ABORT);
  return (jlong)cap;
}

/* Encodes n pieces held back to back in `in` (direct buffer, position 0):
 * piece i = words [segWordOff[i], segWordOff[i+1]).  Writes the packed stream
 * to `out` (direct) and the piece offsets to outOff[n+1].  Same bytes as n
 * PackedOutputStream.write calls (PackedOutputStream.java:35-205). */
JNIEXPORT void JNICALL Java_org_capnproto_gpu_PackedGpu_nativeEncode(
    JNIEnv *env, jclass k, jlong h, jobject in, jlongArray segWordOff, jobject out,
    jlongArray outOff) {
  (void)k;
  void *pin = (*env)->GetDirectBufferAddress(env, in);
  void *pout = (*env)->GetDirectBufferAddress(env, out);
  jlong cap = (*env)->GetDirectBufferCapacity(env, out);
  if (!pin || !pout || !offsets_ok(env, segWordOff) || !outOff ||
      (*env)->GetArrayLength(env, outOff) < (*env)->GetArrayLength(env, segWordOff)) {
    throw_status(env, CPK_EINVAL);
    return;
  }
  jsize n1 = (*env)->GetArrayLength(env, segWordOff);
  jlong *swo = (*env)->GetLongArrayElements(env, segWordOff, NULL);
  if ((uint64_t)(*env)->GetDirectBufferCapacity(env, in) < 8 * (uint64_t)swo[n1 - 1]) {
    (*env)->ReleaseLongArrayElements(env, segWordOff, swo, JNI_ABORT);
    throw_status(env, CPK_EINVAL);
    return;
  }
  jlong *off = (*env)->GetLongArrayElements(env, outOff, NULL);
  int st = cpk_encode_host((cpk_ctx)(intptr_t)h, pin, (const uint64_t *)swo, (uint32_t)(n1 - 1),
                           pout, (uint64_t)cap, (uint64_t *)off);
  (*env)->ReleaseLongArrayElements(env, segWordOff, swo, JNI_ABORT);
  (*env)->ReleaseLongArrayElements(env, outOff, off, 0);
  if (st != CPK_OK) throw_status(env, st);
}

/* Decodes n pieces: piece i's packed bytes are packed[inOff[i]..inOff[i+1])
 * and it fills words [segWordOff[i], segWordOff[i+1]) of `out`.  Throws the
 * first piece's error (DecodeException) like PackedInputStream.read. */
JNIEXPORT void JNICALL Java_org_capnproto_gpu_PackedGpu_nativeDecode(
    JNIEnv *env, jclass k, jlong h, jobject packed, jlongArray inOff, jlongArray segWordOff,
    jobject out) {
  (void)k;
  void *ppk = (*env)->GetDirectBufferAddress(env, packed);
  void *pout = (*env)->GetDirectBufferAddress(env, out);
  if (!ppk || !pout || !offsets_ok(env, segWordOff) || !inOff ||
      (*env)->GetArrayLength(env, inOff) != (*env)->GetArrayLength(env, segWordOff)) {
    throw_status(env, CPK_EINVAL);
    return;
  }
  jsize n1 = (*env)->GetArrayLength(env, segWordOff);
  jlong *swo = (*env)->GetLongArrayElements(env, segWordOff, NULL);
  jlong *io = (*env)->GetLongArrayElements(env, inOff, NULL);
  if ((uint64_t)(*env)->GetDirectBufferCapacity(env, packed) < (uint64_t)io[n1 - 1] ||
      (uint64_t)(*env)->GetDirectBufferCapacity(env, out) < 8 * (uint64_t)swo[n1 - 1]) {
    (*env)->ReleaseLongArrayElements(env, segWordOff, swo, JNI_ABORT);
    (*env)->ReleaseLongArrayElements(env, inOff, io, JNI_ABORT);
    throw_status(env, CPK_EINVAL);
    return;
  }
  int32_t *status = (int32_t *)calloc((size_t)(n1 > 1 ? n1 - 1 : 1), sizeof(int32_t));
  int st = cpk_decode_host((cpk_ctx)(intptr_t)h, ppk, (const uint64_t *)io,
                           (const uint64_t *)swo, (uint32_t)(n1 - 1), pout, status);
  free(status);
  (*env)->ReleaseLongArrayElements(env, segWordOff, swo, JNI_ABORT);
  (*env)->ReleaseLongArrayElements(env, inOff, io, JNI_ABORT);
  if (st != CPK_OK) throw_status(env, st);
}

/* Serialize.write for each message (Serialize.java:256-288): segment i of
 * the batch is words [segWordOff[i], segWordOff[i+1]) of `in` (direct);
 * message m owns segments [msgSegOff[m], msgSegOff[m+1]).  The tables are
 * built on the device.  outOff[nm + nseg + 1]: piece offsets, message order. */
JNIEXPORT void JNICALL Java_org_capnproto_gpu_PackedGpu_nativeEncodeMessages(
    JNIEnv *env, jclass k, jlong h, jobject in, jlongArray segWordOff, jlongArray msgSegOff,
    jobject out, jlongArray outOff) {
  (void)k;
  void *pin = (*env)->GetDirectBufferAddress(env, in);
  void *pout = (*env)->GetDirectBufferAddress(env, out);
  jlong cap = (*env)->GetDirectBufferCapacity(env, out);
  if (!pin || !pout || !offsets_ok(env, segWordOff) || !offsets_ok(env, msgSegOff) || !outOff ||
      (*env)->GetArrayLength(env, outOff) <
          (*env)->GetArrayLength(env, segWordOff) + (*env)->GetArrayLength(env, msgSegOff) - 1) {
    throw_status(env, CPK_EINVAL);
    return;
  }
  jsize ns1 = (*env)->GetArrayLength(env, segWordOff);
  jsize nm1 = (*env)->GetArrayLength(env, msgSegOff);
  jlong *swo = (*env)->GetLongArrayElements(env, segWordOff, NULL);
  jlong *mso = (*env)->GetLongArrayElements(env, msgSegOff, NULL);
  if ((uint64_t)(*env)->GetDirectBufferCapacity(env, in) < 8 * (uint64_t)swo[ns1 - 1]) {
    (*env)->ReleaseLongArrayElements(env, segWordOff, swo, JNI_ABORT);
    (*env)->ReleaseLongArrayElements(env, msgSegOff, mso, JNI_ABORT);
    throw_status(env, CPK_EINVAL);
    return;
  }
  jlong *off = (*env)->GetLongArrayElements(env, outOff, NULL);
  int st = cpk_encode_messages_host((cpk_ctx)(intptr_t)h, pin, (const uint64_t *)swo,
                                    (uint32_t)(ns1 - 1), (const uint64_t *)mso, (uint32_t)(nm1 - 1),
                                    pout, (uint64_t)cap, (uint64_t *)off);
  (*env)->ReleaseLongArrayElements(env, segWordOff, swo, JNI_ABORT);
  (*env)->ReleaseLongArrayElements(env, msgSegOff, mso, JNI_ABORT);
  (*env)->ReleaseLongArrayElements(env, outOff, off, 0);
  if (st != CPK_OK) throw_status(env, st);
}

/* Serialize.read for each message (Serialize.java:119-178): message m is
 * packed[msgOff[m]..msgOff[m+1]).  totals[2] = {words, segments}.  With
 * out == null it only sizes the batch (totals written, no exception); else
 * it fills out, segWordOff[segments+1], msgSegOff[nm+1] and throws the first
 * failed message's error (DecodeException). */
JNIEXPORT void JNICALL Java_org_capnproto_gpu_PackedGpu_nativeDecodeMessages(
    JNIEnv *env, jclass k, jlong h, jobject packed, jlongArray msgOff, jlong traversalLimit,
    jobject out, jlongArray segWordOff, jlongArray msgSegOff, jlongArray totals) {
  (void)k;
  void *ppk = (*env)->GetDirectBufferAddress(env, packed);
  void *pout = out ? (*env)->GetDirectBufferAddress(env, out) : NULL;
  jlong ocap = out ? (*env)->GetDirectBufferCapacity(env, out) : 0;
  if (!ppk || (out && !pout) || !offsets_ok(env, msgOff) || !msgSegOff || !totals ||
      (*env)->GetArrayLength(env, msgSegOff) < (*env)->GetArrayLength(env, msgOff) ||
      (*env)->GetArrayLength(env, totals) < 2) {
    throw_status(env, CPK_EINVAL);
    return;
  }
  jsize nm1 = (*env)->GetArrayLength(env, msgOff);
  jsize sw1 = segWordOff ? (*env)->GetArrayLength(env, segWordOff) : 0;
  jlong *mo = (*env)->GetLongArrayElements(env, msgOff, NULL);
  if ((uint64_t)(*env)->GetDirectBufferCapacity(env, packed) < (uint64_t)mo[nm1 - 1]) {
    (*env)->ReleaseLongArrayElements(env, msgOff, mo, JNI_ABORT);
    throw_status(env, CPK_EINVAL);
    return;
  }
  jlong *ms = (*env)->GetLongArrayElements(env, msgSegOff, NULL);
  jlong *sw = segWordOff ? (*env)->GetLongArrayElements(env, segWordOff, NULL) : NULL;
  jlong *tot = (*env)->GetLongArrayElements(env, totals, NULL);
  int32_t *mst = (int32_t *)calloc((size_t)(nm1 > 1 ? nm1 - 1 : 1), sizeof(int32_t));
  int st = cpk_decode_messages_host((cpk_ctx)(intptr_t)h, ppk, (const uint64_t *)mo,
                                    (uint32_t)(nm1 - 1), (uint64_t)traversalLimit, pout,
                                    (uint64_t)ocap / 8, (uint64_t *)sw,
                                    (uint32_t)(sw1 > 0 ? sw1 - 1 : 0), (uint64_t *)ms, mst,
                                    (uint64_t *)tot);
  free(mst);
  if (sw) (*env)->ReleaseLongArrayElements(env, segWordOff, sw, 0);
  (*env)->ReleaseLongArrayElements(env, msgOff, mo, JNI_ABORT);
  (*env)->ReleaseLongArrayElements(env, msgSegOff, ms, 0);
  (*env)->ReleaseLongArrayElements(env, totals, tot, 0);
  if (st != CPK_OK && !(out == NULL && st == CPK_ENOMEM)) throw_status(env, st);
}

/* long PackedGpu.nativeDecodeStream(long h, ByteBuffer packed, long[] segWordOff,
 *                                   ByteBuffer out)
 * read() calls back to back on one packed stream (PackedInputStream.java:
 * 35-140, as fillBuffer issues them, Serialize.java:74-83): piece i fills
 * words [segWordOff[i], segWordOff[i+1]) of `out`, each consuming only the
 * bytes it needs.  The stream is packed[position, limit) (direct).  Returns
 * the bytes consumed; throws the first failed piece's error. */
JNIEXPORT jlong JNICALL Java_org_capnproto_gpu_PackedGpu_nativeDecodeStream(
    JNIEnv *env, jclass k, jlong h, jobject packed, jint position, jint limit,
    jlongArray segWordOff, jobject out) {
  (void)k;
  uint8_t *ppk = (uint8_t *)(*env)->GetDirectBufferAddress(env, packed);
  void *pout = (*env)->GetDirectBufferAddress(env, out);
  if (!ppk || !pout || position < 0 || limit < position || !offsets_ok(env, segWordOff) ||
      (*env)->GetDirectBufferCapacity(env, packed) < limit) {
    throw_status(env, CPK_EINVAL);
    return 0;
  }
  jsize n1 = (*env)->GetArrayLength(env, segWordOff);
  uint32_t n = (uint32_t)(n1 - 1);
  jlong *swo = (*env)->GetLongArrayElements(env, segWordOff, NULL);
  if ((uint64_t)(*env)->GetDirectBufferCapacity(env, out) < 8 * (uint64_t)swo[n]) {
    (*env)->ReleaseLongArrayElements(env, segWordOff, swo, JNI_ABORT);
    throw_status(env, CPK_EINVAL);
    return 0;
  }
  uint64_t *in_off = (uint64_t *)calloc((size_t)n + 1, sizeof(uint64_t));
  int32_t *status = (int32_t *)calloc((size_t)(n ? n : 1), sizeof(int32_t));
  int st = (in_off && status)
               ? cpk_decode_stream_host((cpk_ctx)(intptr_t)h, ppk + position,
                                        (uint64_t)(limit - position), (const uint64_t *)swo, n,
                                        pout, in_off, status)
               : CPK_ENOMEM;
  jlong used = (st == CPK_OK) ? (jlong)in_off[n] : 0;
  free(in_off);
  free(status);
  (*env)->ReleaseLongArrayElements(env, segWordOff, swo, JNI_ABORT);
  if (st != CPK_OK) throw_status(env, st);
  return used;
}

/* void PackedGpu.nativeEncodeGather(long h, ByteBuffer[] pieces, int[] positions,
 *                                   long[] segWordOff, ByteBuffer out, long[] outOff)
 * Zero-copy encode of direct buffers where they lie (SURVEY.md §8f row 4;
 * builder segments allocated DIRECT, DefaultAllocator.java:56-62): piece i is
 * pieces[i][positions[i], +8*(segWordOff[i+1]-segWordOff[i])) ->
 * cpk_encode_host_gather.  Same bytes as nativeEncode over the concatenation. */
JNIEXPORT void JNICALL Java_org_capnproto_gpu_PackedGpu_nativeEncodeGather(
    JNIEnv *env, jclass k, jlong h, jobjectArray pieces, jintArray positions,
    jlongArray segWordOff, jobject out, jlongArray outOff) {
  (void)k;
  void *pout = (*env)->GetDirectBufferAddress(env, out);
  jlong cap = (*env)->GetDirectBufferCapacity(env, out);
  jsize n = pieces ? (*env)->GetArrayLength(env, pieces) : -1;
  if (!pout || n < 0 || !positions || (*env)->GetArrayLength(env, positions) != n || !segWordOff ||
      (*env)->GetArrayLength(env, segWordOff) != n + 1 || !outOff ||
      (*env)->GetArrayLength(env, outOff) < n + 1) {
    throw_status(env, CPK_EINVAL);
    return;
  }
  const void **ptrs = (const void **)calloc((size_t)(n ? n : 1), sizeof(void *));
  if (!ptrs) {
    throw_status(env, CPK_ENOMEM);
    return;
  }
  jlong *swo = (*env)->GetLongArrayElements(env, segWordOff, NULL);
  jint *pos = (*env)->GetIntArrayElements(env, positions, NULL);
  int st = CPK_OK;
  for (jsize i = 0; i < n && st == CPK_OK; ++i) {
    if (swo[i + 1] < swo[i]) {
      st = CPK_EINVAL;
      break;
    }
    jobject b = (*env)->GetObjectArrayElement(env, pieces, i);
    ptrs[i] = gather_ptr(env, b, pos[i], 8 * (uint64_t)(swo[i + 1] - swo[i]), &st);
    if (b) (*env)->DeleteLocalRef(env, b);
  }
  (*env)->ReleaseIntArrayElements(env, positions, pos, JNI_ABORT);
  jlong *off = (*env)->GetLongArrayElements(env, outOff, NULL);
  if (st == CPK_OK)
    st = cpk_encode_host_gather((cpk_ctx)(intptr_t)h, ptrs, (const uint64_t *)swo, (uint32_t)n,
                                pout, (uint64_t)cap, (uint64_t *)off);
  free(ptrs);
  (*env)->ReleaseLongArrayElements(env, segWordOff, swo, JNI_ABORT);
  (*env)->ReleaseLongArrayElements(env, outOff, off, st == CPK_OK ? 0 : JNI_ABORT);
  if (st != CPK_OK) throw_status(env, st);
}

/* void PackedGpu.nativeEncodeMessagesGather(long h, ByteBuffer[] segs, int[] positions,
 *     long[] segWordOff, long[] msgSegOff, ByteBuffer out, long[] outOff)
 * nativeEncodeMessages with every segment a direct buffer packed where it
 * lies (cpk_encode_messages_host_gather; builder segments allocated DIRECT,
 * DefaultAllocator.java:56-62). */
JNIEXPORT void JNICALL Java_org_capnproto_gpu_PackedGpu_nativeEncodeMessagesGather(
    JNIEnv *env, jclass k, jlong h, jobjectArray segs, jintArray positions, jlongArray segWordOff,
    jlongArray msgSegOff, jobject out, jlongArray outOff) {
  (void)k;
  void *pout = (*env)->GetDirectBufferAddress(env, out);
  jlong cap = (*env)->GetDirectBufferCapacity(env, out);
  jsize ns = segs ? (*env)->GetArrayLength(env, segs) : -1;
  if (!pout || ns < 0 || !positions || (*env)->GetArrayLength(env, positions) != ns || !segWordOff ||
      (*env)->GetArrayLength(env, segWordOff) != ns + 1 || !offsets_ok(env, msgSegOff) || !outOff ||
      (*env)->GetArrayLength(env, outOff) < ns + (*env)->GetArrayLength(env, msgSegOff)) {
    throw_status(env, CPK_EINVAL);
    return;
  }
  const void **ptrs = (const void **)calloc((size_t)(ns ? ns : 1), sizeof(void *));
  if (!ptrs) {
    throw_status(env, CPK_ENOMEM);
    return;
  }
  jlong *swo = (*env)->GetLongArrayElements(env, segWordOff, NULL);
  jint *pos = (*env)->GetIntArrayElements(env, positions, NULL);
  int st = CPK_OK;
  for (jsize i = 0; i < ns && st == CPK_OK; ++i) {
    if (swo[i + 1] < swo[i]) {
      st = CPK_EINVAL;
      break;
    }
    jobject b = (*env)->GetObjectArrayElement(env, segs, i);
    ptrs[i] = gather_ptr(env, b, pos[i], 8 * (uint64_t)(swo[i + 1] - swo[i]), &st);
    if (b) (*env)->DeleteLocalRef(env, b);
  }
  (*env)->ReleaseIntArrayElements(env, positions, pos, JNI_ABORT);
  jsize nm1 = (*env)->GetArrayLength(env, msgSegOff);
  jlong *mso = (*env)->GetLongArrayElements(env, msgSegOff, NULL);
  jlong *off = (*env)->GetLongArrayElements(env, outOff, NULL);
  if (st == CPK_OK)
    st = cpk_encode_messages_host_gather((cpk_ctx)(intptr_t)h, ptrs, (const uint64_t *)swo,
                                         (uint32_t)ns, (const uint64_t *)mso, (uint32_t)(nm1 - 1),
                                         pout, (uint64_t)cap, (uint64_t *)off);
  free(ptrs);
  (*env)->ReleaseLongArrayElements(env, segWordOff, swo, JNI_ABORT);
  (*env)->ReleaseLongArrayElements(env, msgSegOff, mso, JNI_ABORT);
  (*env)->ReleaseLongArrayElements(env, outOff, off, st == CPK_OK ? 0 : JNI_ABORT);
  if (st != CPK_OK) throw_status(env, st);
}

/* int PackedGpu.nativeReadMessage(long h, ByteBuffer packed, int position, int limit,
 *                                 long traversalLimit, ByteBuffer out, long[] info)
 * SerializePacked.read of one message from packed[position, limit) (direct)
 * in one library call (cpk_read_message_host: table read and checked, every
 * segment decoded, Serialize.java:119-178).  out (direct) gets the segments
 * back to back; info[CPK_MSG_INFO_WORDS] = status, bytes consumed, segment
 * count, words, segment word offsets.  Returns CPK_OK, or -- without
 * throwing -- CPK_ETRUNC (the bytes end inside the message: the caller takes
 * more) and CPK_ENOMEM with info[3] = the words needed (out too small); any
 * other status throws (DecodeException for a malformed message). */
JNIEXPORT jint JNICALL Java_org_capnproto_gpu_PackedGpu_nativeReadMessage(
    JNIEnv *env, jclass k, jlong h, jobject packed, jint position, jint limit, jlong traversalLimit,
    jobject out, jlongArray info) {
  (void)k;
  uint8_t *ppk = (uint8_t *)(*env)->GetDirectBufferAddress(env, packed);
  void *pout = (*env)->GetDirectBufferAddress(env, out);
  jlong ocap = pout ? (*env)->GetDirectBufferCapacity(env, out) : -1;
  if (!ppk || !pout || ocap < 0 || position < 0 || limit < position ||
      (*env)->GetDirectBufferCapacity(env, packed) < limit || !info ||
      (*env)->GetArrayLength(env, info) < CPK_MSG_INFO_WORDS) {
    throw_status(env, CPK_EINVAL);
    return CPK_EINVAL;
  }
  uint64_t row[CPK_MSG_INFO_WORDS];
  memset(row, 0, sizeof row);
  int st = cpk_read_message_host((cpk_ctx)(intptr_t)h, ppk + position, (uint64_t)(limit - position),
                                 (uint64_t)traversalLimit, pout, (uint64_t)ocap / 8, row);
  (*env)->SetLongArrayRegion(env, info, 0, CPK_MSG_INFO_WORDS, (const jlong *)row);
  if (st == CPK_ENOMEM && (int64_t)row[0] != CPK_ENOMEM) {  /* (a real allocation failure) */
    throw_status(env, st);
    return st;
  }
  if (st != CPK_OK && st != CPK_ETRUNC && st != CPK_ENOMEM) throw_status(env, st);
  return st;
}
