package org.apache.spark.ml.feature.languagedetection

import java.nio.{ByteBuffer, ByteOrder}
import java.util.concurrent.ConcurrentHashMap

/**
  * JNI bindings of libldgpu.so (include/ldgpu.h) through libldgpu_jni.so
  * (jni/ldgpu_jni.c).  Every buffer argument is a DIRECT ByteBuffer in native
  * byte order; handles are the C pointers as Longs.  A non-zero status turns
  * into the JVM exception the reference raises for the same condition
  * (LdgpuNative.check).
  *
  * Per executor JVM: one context per device and one device table per
  * broadcast table (LanguageDetectorModel.scala:222 broadcasts the map once
  * per transform), shared by the executor's task threads -- every C entry
  * point is thread-safe and concurrent scoring calls run on their own
  * streams.
  */
object LdgpuNative {
  System.loadLibrary("ldgpu_jni")

  // ---- C ABI (status codes of enum ldgpu_status)
  val OK = 0
  val EINVAL = 1
  val EROWLEN = 2
  val ENOMEM = 3
  val EDEVICE = 4
  val EUNSUPPORTED = 5
  val ENODEV = 6

  @native def lastError(): String
  @native def ctxCreate(device: Int, out: Array[Long]): Int
  @native def hostAlloc(ctx: Long, bytes: Long): ByteBuffer          // pinned, direct; null on failure
  @native def hostFree(ctx: Long, buf: ByteBuffer): Int
  @native def modelCreate(ctx: Long, nRows: Long, keyBytes: ByteBuffer, keyOffsets: ByteBuffer, rows: ByteBuffer,
                          rowOk: ByteBuffer, nLangs: Int, gramLengths: Array[Int], out: Array[Long]): Int
  /** mask form: row i = vals(i) at the languages set in masks [nRows][ceil(nLangs / 64)] */
  @native def modelCreateMasks(ctx: Long, nRows: Long, keyBytes: ByteBuffer, keyOffsets: ByteBuffer,
                               masks: ByteBuffer, vals: ByteBuffer, nLangs: Int, gramLengths: Array[Int],
                               out: Array[Long]): Int
  @native def modelDestroy(model: Long): Int
  /** nLangs: the model's languages (the shim checks a non-null scores buffer's capacity with it) */
  @native def score(model: Long, bytes: ByteBuffer, offsets: ByteBuffer, nDocs: Long, labels: ByteBuffer,
                    scores: ByteBuffer, nLangs: Int): Int
  @native def countsCreate(ctx: Long, nLangs: Int, gramLengths: Array[Int], capacityHint: Long,
                           out: Array[Long]): Int
  @native def countsDestroy(counts: Long): Int
  @native def count(counts: Long, bytes: ByteBuffer, offsets: ByteBuffer, docLang: ByteBuffer, nDocs: Long): Int
  /** out(0) = distinct grams, out(1) = their total key bytes */
  @native def countsSize(counts: Long, out: Array[Long]): Int
  @native def countsExport(counts: Long, keyBytes: ByteBuffer, keyOffsets: ByteBuffer, counts_ : ByteBuffer,
                           nLangs: Int): Int
  @native def countsAdd(counts: Long, n: Long, keyBytes: ByteBuffer, keyOffsets: ByteBuffer, rows: ByteBuffer,
                        nLangs: Int): Int
  /** grams [first, first + n) of the (length, bytes) order: out(0) = key bytes, out(1) = (language, count) pairs */
  @native def countsSparseSize(counts: Long, first: Long, n: Long, out: Array[Long]): Int
  @native def countsExportSparse(counts: Long, first: Long, n: Long, keyBytes: ByteBuffer, keyOffsets: ByteBuffer,
                                 pairOffsets: ByteBuffer, pairLangs: ByteBuffer, pairCounts: ByteBuffer): Int
  @native def countsAddSparse(counts: Long, n: Long, keyBytes: ByteBuffer, keyOffsets: ByteBuffer,
                              pairOffsets: ByteBuffer, pairLangs: ByteBuffer, pairCounts: ByteBuffer): Int
  /** out(0) = table rows, out(1) = their total key bytes */
  @native def fitTableSize(counts: Long, profileSize: Int, out: Array[Long]): Int
  @native def fitTableExport(counts: Long, keyBytes: ByteBuffer, keyOffsets: ByteBuffer, rows: ByteBuffer,
                             nRows: Long, keyBytesN: Long, nLangs: Int): Int
  @native def fitTableExportMasks(counts: Long, keyBytes: ByteBuffer, keyOffsets: ByteBuffer, masks: ByteBuffer,
                                  vals: ByteBuffer, nRows: Long, keyBytesN: Long, nLangs: Int): Int
  // multi-GPU merge (Spark with barrier execution: one task per GPU)
  @native def commUniqueId(): Array[Byte]
  @native def commCreateRccl(ctx: Long, id: Array[Byte], rank: Int, world: Int, out: Array[Long]): Int
  @native def commDestroy(comm: Long): Int
  @native def countsMerge(counts: Long, comm: Long): Int
  // the preprocessors on the device (include/ldgpu.h PREPROCESS)
  /** lower: 65536 u16, Character.toLowerCase of every unit; special: 8192 bytes, bit u = unit u goes to the host */
  @native def casemapCreate(ctx: Long, lower: ByteBuffer, special: ByteBuffer, out: Array[Long]): Int
  @native def casemapDestroy(map: Long): Int
  /** units: UTF-16 code units, offsets in units; out: offsets(nDocs) - offsets(0) units (bytes with PreLowBytes);
    * outOffsets: nDocs + 1 longs; host, locale (nullable): nDocs bytes */
  @native def preprocess(map: Long, units: ByteBuffer, offsets: ByteBuffer, nDocs: Long, locale: ByteBuffer,
                         flags: Int, out: ByteBuffer, outOffsets: ByteBuffer, host: ByteBuffer): Int

  val PreLower = 1
  val PreClean = 2
  val PreLowBytes = 4
  val LocaleRoot = 0
  val LocaleTrAz = 1
  val LocaleLt = 2

  /** The reference's exception for each failure class: a wrong-length row
    * hit (BLAS.axpy's require) and n <= 0 (sliding's require) are
    * IllegalArgumentException, allocation failures OutOfMemoryError. */
  def check(status: Int): Unit = status match {
    case OK => ()
    case EINVAL | EROWLEN => throw new IllegalArgumentException(lastError())
    case ENOMEM => throw new OutOfMemoryError(lastError())
    case EUNSUPPORTED => throw new UnsupportedOperationException(lastError())
    case _ => throw new RuntimeException(s"libldgpu: ${lastError()}")
  }

  /** A JVM direct buffer holds at most Int.MaxValue bytes: larger requests
    * fail here (callers export / import in ranges that stay below it) instead
    * of wrapping to a small or negative size. */
  val MaxDirect: Long = Int.MaxValue.toLong

  def direct(bytes: Long): ByteBuffer = {
    if (bytes < 0L || bytes > MaxDirect)
      throw new IllegalArgumentException(s"a direct buffer of $bytes bytes is outside [0, $MaxDirect]")
    ByteBuffer.allocateDirect(math.max(bytes, 1L).toInt).order(ByteOrder.nativeOrder())
  }

  /** The executor's GPU: executors are pinned one per GPU (HIP_VISIBLE_DEVICES),
    * so device 0 unless LDGPU_DEVICE says otherwise. */
  def defaultDevice: Int = sys.env.get("LDGPU_DEVICE").map(_.toInt).getOrElse(0)

  private val contexts = new ConcurrentHashMap[Integer, java.lang.Long]()

  def context(device: Int = defaultDevice): Long = {
    val have = contexts.get(device)
    if (have != null) have.longValue
    else contexts.synchronized {
      val again = contexts.get(device)
      if (again != null) again.longValue
      else {
        val out = new Array[Long](1)
        check(ctxCreate(device, out))
        contexts.put(device, out(0))
        out(0)
      }
    }
  }

  // Device tables of this executor, keyed by the broadcast that carries them,
  // least recently used first.  A transform creates a new broadcast, so the
  // cache is bounded: at most maxModels tables (and maxModelBytes of their
  // uploaded host form) stay on the GPU, the least recently used is freed
  // first -- never one a running task still scores with (refs > 0).
  var maxModels: Int = 4
  var maxModelBytes: Long = 8L << 30

  private final class Entry(val handle: Long, val bytes: Long) {
    var refs: Int = 0
  }

  private val models = new java.util.LinkedHashMap[java.lang.Long, Entry](16, 0.75f, true)

  /** The device table of a broadcast, uploaded on first use; pair every call
    * with releaseModel(broadcastId) once the task is done scoring. */
  def acquireModel(broadcastId: Long, table: PackedTable, gramLengths: Array[Int]): Long = models.synchronized {
    val have = models.get(broadcastId)
    val e = if (have != null) have else {
      val fresh = new Entry(table.upload(context(), gramLengths), table.hostBytes)
      models.put(broadcastId, fresh)
      evict(broadcastId)
      fresh
    }
    e.refs += 1
    e.handle
  }

  def releaseModel(broadcastId: Long): Unit = models.synchronized {
    val e = models.get(broadcastId)
    if (e != null) {
      e.refs -= 1
      evict(-1L)
    }
  }

  /** Drop a broadcast's table at once (when the broadcast is destroyed). */
  def forgetModel(broadcastId: Long): Unit = models.synchronized {
    val e = models.get(broadcastId)
    if (e != null && e.refs <= 0) {
      models.remove(broadcastId)
      modelDestroy(e.handle)
    }
  }

  // least recently used first, skipping tables in use and `keep`
  private def evict(keep: Long): Unit = {
    var bytes = 0L
    val it0 = models.values().iterator()
    while (it0.hasNext) bytes += it0.next().bytes
    val it = models.entrySet().iterator()
    while (it.hasNext && (models.size > maxModels || bytes > maxModelBytes)) {
      val kv = it.next()
      val e = kv.getValue
      if (e.refs <= 0 && kv.getKey.longValue != keep) {
        it.remove()
        bytes -= e.bytes
        modelDestroy(e.handle)
      }
    }
  }
}
