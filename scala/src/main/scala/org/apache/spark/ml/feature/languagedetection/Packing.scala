package org.apache.spark.ml.feature.languagedetection

import java.nio.ByteBuffer
import java.nio.charset.StandardCharsets

/**
  * The gram -> probability-row map as the flat arrays ldgpu_model_create
  * takes: key bytes + offsets, dense rows [n][nLangs] in supported-language
  * order, and a row-length flag.  transform broadcasts this (one array per
  * field) instead of a Map of boxed Seq[Byte] keys.
  *
  * A row whose length differs from the number of languages is kept with
  * rowOk = 0: a document that hits it fails as BLAS.axpy's size check does
  * (LanguageDetectorModel.scala:148-149), one that does not hit it scores.
  */
case class PackedTable(keyBytes: Array[Byte], keyOffsets: Array[Long], rows: Array[Double], rowOk: Array[Byte],
                       nLangs: Int) {
  def nRows: Int = keyOffsets.length - 1

  /** a device table on `ctx` (the executor's GPU) */
  def upload(ctx: Long, gramLengths: Array[Int]): Long = {
    val kb = LdgpuNative.direct(keyBytes.length.toLong)
    kb.put(keyBytes).flip()
    val ko = LdgpuNative.direct(8L * keyOffsets.length)
    ko.asLongBuffer().put(keyOffsets)
    val rw = LdgpuNative.direct(8L * rows.length)
    rw.asDoubleBuffer().put(rows)
    val ok = LdgpuNative.direct(rowOk.length.toLong)
    ok.put(rowOk).flip()
    val out = new Array[Long](1)
    LdgpuNative.check(LdgpuNative.modelCreate(ctx, nRows.toLong, kb, ko, rw, ok, nLangs, gramLengths, out))
    out(0)
  }
}

object PackedTable {
  def of(map: Map[Seq[Byte], Array[Double]], nLangs: Int): PackedTable = {
    val entries = map.toArray
    val offsets = new Array[Long](entries.length + 1)
    var i = 0
    while (i < entries.length) {
      offsets(i + 1) = offsets(i) + entries(i)._1.length
      i += 1
    }
    val keys = new Array[Byte](offsets(entries.length).toInt)
    val rows = new Array[Double](entries.length * nLangs)
    val ok = new Array[Byte](entries.length)
    i = 0
    while (i < entries.length) {
      val (k, row) = entries(i)
      k.copyToArray(keys, offsets(i).toInt)
      if (row.length == nLangs) {
        System.arraycopy(row, 0, rows, i * nLangs, nLangs)
        ok(i) = 1
      }
      i += 1
    }
    PackedTable(keys, offsets, rows, ok, nLangs)
  }
}

/**
  * One batch of a partition's documents packed for the C ABI: bytes, int64
  * offsets, int32 language ids (FIT) and int32 labels (SCORE), all direct
  * buffers reused across batches.  Buffers come from ldgpu_host_alloc (pinned
  * host memory) when a context is given, so the library copies them to the
  * GPU without a staging copy.  A batch is full at maxDocs documents or
  * targetBytes bytes (a single larger document grows the byte buffer).
  */
final class DocBatch(ctx: Long, maxDocs: Int, targetBytes: Int) {
  private val pinned = new java.util.IdentityHashMap[ByteBuffer, java.lang.Boolean]()

  private def alloc(bytes: Long): ByteBuffer = {
    val b = if (ctx != 0L) LdgpuNative.hostAlloc(ctx, bytes) else null
    if (b != null) {
      pinned.put(b, java.lang.Boolean.TRUE)
      b.order(java.nio.ByteOrder.nativeOrder())
    } else {
      LdgpuNative.direct(bytes)
    }
  }

  private var byteCap = math.max(targetBytes, 1 << 16)
  var bytes: ByteBuffer = alloc(byteCap.toLong + 16)
  val offsets: ByteBuffer = alloc(8L * (maxDocs + 1))
  val langs: ByteBuffer = alloc(4L * maxDocs)
  val labels: ByteBuffer = alloc(4L * maxDocs)
  var n = 0
  var used = 0

  def clear(): Unit = {
    n = 0
    used = 0
    offsets.putLong(0, 0L)
  }

  def full: Boolean = n == maxDocs || used >= targetBytes

  private def ensure(extra: Int): Unit = if (used.toLong + extra > byteCap) {
    val grown = alloc(math.max(2L * byteCap, used.toLong + extra) + 16)
    val old = bytes.duplicate()
    old.position(0).limit(used)
    grown.put(old)
    free(bytes)
    bytes = grown
    byteCap = grown.capacity() - 16
  }

  private def push(b: Array[Byte], lang: Int): Unit = {
    ensure(b.length)
    var j = 0
    while (j < b.length) {
      bytes.put(used + j, b(j))
      j += 1
    }
    used += b.length
    langs.putInt(4 * n, lang)
    n += 1
    offsets.putLong(8 * n, used.toLong)
  }

  /** SCORE encoding: the low byte of every UTF-16 code unit, as
    * detect(String, ...) does (LanguageDetectorModel.scala:161).  A null text
    * throws NullPointerException there too. */
  def addScore(text: String): Unit = {
    val len = text.length
    val b = new Array[Byte](len)
    var j = 0
    while (j < len) {
      b(j) = text.charAt(j).toByte
      j += 1
    }
    push(b, 0)
  }

  /** FIT encoding: String.getBytes(UTF-8) (LanguageDetector.scala:37; a lone
    * surrogate becomes '?'); lang = index in supportedLanguages or -1 */
  def addFit(text: String, lang: Int): Unit = push(text.getBytes(StandardCharsets.UTF_8), lang)

  def label(i: Int): Int = labels.getInt(4 * i)

  private def free(b: ByteBuffer): Unit = if (b != null && pinned.remove(b) != null) LdgpuNative.hostFree(ctx, b)

  def close(): Unit = Seq(bytes, offsets, langs, labels).foreach(free)
}
