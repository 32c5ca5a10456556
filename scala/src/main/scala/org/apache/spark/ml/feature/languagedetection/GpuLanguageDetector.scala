package org.apache.spark.ml.feature.languagedetection

import java.nio.charset.StandardCharsets.ISO_8859_1

import org.apache.spark.internal.Logging
import org.apache.spark.ml.Estimator
import org.apache.spark.ml.param.shared.{HasInputCol, HasLabelCol}
import org.apache.spark.ml.param.{Param, ParamMap}
import org.apache.spark.ml.util.Identifiable
import org.apache.spark.sql.types.StructType
import org.apache.spark.sql.{Dataset, SaveMode}

/**
  * Drop-in for the reference's LanguageDetector Estimator (same package, class
  * name, constructors, params, defaults, validation messages and order;
  * LanguageDetector.scala:176-264).  The counting runs on the executors' GPUs
  * (libldgpu.so), see LanguageDetector.computeGramProbabilities.
  */
class LanguageDetector(val uid: String,
                       val supportedLanguages: Seq[String],
                       val gramLengths: Seq[Int],
                       val languageProfileSize: Int)
  extends Estimator[LanguageDetectorModel] with HasInputCol with HasLabelCol {

  def this(supportedLanguages: Seq[String], gramLengths: Seq[Int], languageProfileSize: Int) =
    this(Identifiable.randomUID("LanguageDetector"), supportedLanguages, gramLengths, languageProfileSize)

  setDefault(inputCol -> "fulltext", labelCol -> "lang")

  def setInputCol(value: String): this.type = set(inputCol, value)
  def setLabelCol(value: String): this.type = set(labelCol, value)

  val saveGramsToHDFS = new Param[Option[String]](this, "saveGrams", "Persist the dataset of grams to HDFS")
  def setSaveGramsToHDFS(value: Option[String]): this.type = set(saveGramsToHDFS, value)
  setDefault(saveGramsToHDFS -> None)

  override def transformSchema(schema: StructType): StructType = schema

  override def copy(extra: ParamMap): LanguageDetector =
    copyValues(new LanguageDetector(uid, supportedLanguages, gramLengths, languageProfileSize), extra)

  override def fit(dataset: Dataset[_]): LanguageDetectorModel = {
    import dataset.sparkSession.implicits._
    val data = dataset.select($(labelCol), $(inputCol)).as[(String, String)].cache()
    // the reference's checks, in its order (LanguageDetector.scala:221-238):
    // an unsupported label first (raised inside a job), then a supported
    // language without rows -- one distinct-labels job serves both
    val supported = supportedLanguages.toSet
    val labels = data.map(_._1).distinct()
    labels.foreach { lang =>
      if (!supported.contains(lang))
        throw new Exception(s"Input data contians $lang, but it is not in the list of supported languages")
    }
    val present = labels.collect().toSet
    supportedLanguages.foreach { lang =>
      if (!present.contains(lang))
        throw new Exception(s"No training examples found for language $lang. Provide examples for each language")
    }
    val probabilities =
      LanguageDetector.computeGramProbabilities(data, gramLengths, languageProfileSize, supportedLanguages).cache()
    $(saveGramsToHDFS).foreach(path => LanguageDetector.save(path, probabilities))
    val table = probabilities.collect().toMap
    data.unpersist()
    probabilities.unpersist()
    new LanguageDetectorModel(table, gramLengths, supportedLanguages)
  }
}

/** One gram's nonzero (language, count) pairs, languages ascending: the sparse
  * row of the count table that crosses the shuffle (~1.3 pairs per gram on
  * the fit corpora against nLangs dense Longs). */
final case class SparseCounts(langs: Array[Int], counts: Array[Long]) {
  /** the sum of two rows (a merge of the two sorted language lists) */
  def +(o: SparseCounts): SparseCounts = {
    val l = new Array[Int](langs.length + o.langs.length)
    val c = new Array[Long](l.length)
    var (i, j, k) = (0, 0, 0)
    while (i < langs.length || j < o.langs.length) {
      if (j == o.langs.length || (i < langs.length && langs(i) < o.langs(j))) {
        l(k) = langs(i); c(k) = counts(i); i += 1
      } else if (i == langs.length || o.langs(j) < langs(i)) {
        l(k) = o.langs(j); c(k) = o.counts(j); j += 1
      } else {
        l(k) = langs(i); c(k) = counts(i) + o.counts(j); i += 1; j += 1
      }
      k += 1
    }
    SparseCounts(java.util.Arrays.copyOf(l, k), java.util.Arrays.copyOf(c, k))
  }
}

object LanguageDetector extends Logging {

  /** documents / bytes per ldgpu_count call */
  var batchDocs: Int = 1 << 20
  var batchBytes: Int = 64 << 20
  /** grams per ranged sparse export / import (each range's buffers stay < 2 GiB) */
  var rangeGrams: Long = 1L << 20

  /**
    * computeGramProbabilities (LanguageDetector.scala:145-165) on the GPUs:
    *  1. every partition counts its rows on its executor's GPU (ldgpu_count:
    *     computeGrams + reduceGrams for the partition) and emits one row per
    *     distinct gram: (key, its nonzero (language, count) pairs);
    *  2. one shuffle sums those sparse rows per gram (integer sums: the
    *     reference's counts, bit-exact) -- instead of the reference's L + 1
    *     shuffles of every window record;
    *  3. every partition of the global rows -- each gram in exactly one, with
    *     its global counts, hence its global presence class -- builds its own
    *     top-K table on its GPU (ldgpu_fit_table_size): per language the K best
    *     by (value, then (length, bytes)), which holds every gram of the global
    *     top-K that lives in the partition; it leaves in mask form (key, mask
    *     words, value);
    *  4. the driver keeps, per language, the K best candidates (same order).
    * Ties follow the build's deterministic (length, unsigned bytes) rule where
    * the reference's follow Spark's shuffle order (DESIGN.md, stated
    * divergences); every result satisfies the reference's top-K contract.
    * On Spark with barrier execution, steps 2-4 can instead run inside the
    * library over RCCL (LdgpuNative.countsMerge; INTEGRATION.md).
    */
  def computeGramProbabilities(data: Dataset[(String, String)],
                               gramLengths: Seq[Int],
                               languageProfileSize: Int,
                               supportedLanguages: Seq[String]): Dataset[(Seq[Byte], Array[Double])] = {
    val spark = data.sparkSession
    import spark.implicits._
    val nLangs = supportedLanguages.length
    val index = supportedLanguages.zipWithIndex.toMap
    val grams = gramLengths.toArray
    val (docs, bytes, range) = (batchDocs, batchBytes, rangeGrams)
    val counted = data.rdd.mapPartitions(it => countPartition(it, index, nLangs, grams, docs, bytes, range))
    val global = counted.reduceByKey(_ + _)
    val candidates = global.mapPartitions(it => partitionTopK(it, nLangs, grams, languageProfileSize, range))
    val table = selectTopK(candidates.collect(), nLangs, languageProfileSize)
    spark.createDataset(table.toSeq)
  }

  private def countPartition(it: Iterator[(String, String)], index: Map[String, Int], nLangs: Int,
                             grams: Array[Int], docs: Int, bytes: Int,
                             range: Long): Iterator[(String, SparseCounts)] = {
    if (!it.hasNext) return Iterator.empty
    val ctx = LdgpuNative.context()
    val out = new Array[Long](1)
    LdgpuNative.check(LdgpuNative.countsCreate(ctx, nLangs, grams, 0L, out))
    val counts = out(0)
    val batch = new DocBatch(ctx, docs, bytes)
    try {
      while (it.hasNext) {
        batch.clear()
        while (it.hasNext && !batch.full) {
          val (lang, text) = it.next()
          batch.addFit(text, index.getOrElse(lang, -1))  // rows of other languages are skipped, as reduceGrams does
        }
        LdgpuNative.check(LdgpuNative.count(counts, batch.bytes, batch.offsets, batch.langs, batch.n.toLong))
      }
    } catch {
      case e: Throwable =>
        LdgpuNative.countsDestroy(counts)
        throw e
    } finally {
      batch.close()
    }
    new CountsExport(counts, range)
  }

  /** (key bytes as an ISO-8859-1 string: one char per byte, a hashable
    * shuffle key; its sparse counts) of every distinct gram of a count table,
    * streamed: one ranged export of at most `range` grams (halved while a
    * range's buffers would pass 1 GiB) is held at a time, its rows built as
    * the shuffle consumes them.  The table is destroyed when the iterator is
    * exhausted or the task ends. */
  private final class CountsExport(counts: Long, range: Long) extends Iterator[(String, SparseCounts)] {
    private var open = true
    private val total: Long = {
      val size = new Array[Long](2)
      LdgpuNative.check(LdgpuNative.countsSize(counts, size))
      size(0)
    }
    private var first = 0L
    private var n = 0L
    private var i = 0L
    private var kb, ko, po, pl, pc: java.nio.ByteBuffer = _
    Option(org.apache.spark.TaskContext.get()).foreach(_.addTaskCompletionListener { _: org.apache.spark.TaskContext =>
      close()
    })

    private def close(): Unit = if (open) {
      open = false
      LdgpuNative.countsDestroy(counts)
    }

    private def load(): Unit = {
      n = math.min(range, total - first)
      val sz = new Array[Long](2)
      LdgpuNative.check(LdgpuNative.countsSparseSize(counts, first, n, sz))
      while (n > 1 && (sz(0) > (1L << 30) || 8L * sz(1) > (1L << 30) || 8L * (n + 1) > (1L << 30))) {
        n = n / 2
        LdgpuNative.check(LdgpuNative.countsSparseSize(counts, first, n, sz))
      }
      kb = LdgpuNative.direct(sz(0))
      ko = LdgpuNative.direct(8L * (n + 1))
      po = LdgpuNative.direct(8L * (n + 1))
      pl = LdgpuNative.direct(4L * sz(1))
      pc = LdgpuNative.direct(8L * sz(1))
      LdgpuNative.check(LdgpuNative.countsExportSparse(counts, first, n, kb, ko, po, pl, pc))
      first += n
      i = 0
    }

    override def hasNext: Boolean = {
      if (i < n) return true
      if (open && first < total) {
        load()
        return true
      }
      close()
      false
    }

    override def next(): (String, SparseCounts) = {
      if (!hasNext) throw new NoSuchElementException("count table exhausted")
      val (a, b) = (ko.getLong(8 * i.toInt).toInt, ko.getLong(8 * (i.toInt + 1)).toInt)
      val key = new Array[Byte](b - a)
      kb.position(a)
      kb.get(key)
      val (p0, p1) = (po.getLong(8 * i.toInt).toInt, po.getLong(8 * (i.toInt + 1)).toInt)
      val langs = new Array[Int](p1 - p0)
      val cnts = new Array[Long](p1 - p0)
      var j = 0
      while (j < langs.length) {
        langs(j) = pl.getInt(4 * (p0 + j))
        cnts(j) = pc.getLong(8 * (p0 + j))
        j += 1
      }
      i += 1
      (new String(key, ISO_8859_1), SparseCounts(langs, cnts))
    }
  }

  /** the partition's global rows into a device table -- streamed through
    * fixed direct buffers (at most `range` rows, 64 MiB of key bytes and
    * 2^24 pairs per ranged sparse import), never held whole -- and its top-K
    * table out in mask form: (key, mask words, value) */
  private def partitionTopK(it: Iterator[(String, SparseCounts)], nLangs: Int, grams: Array[Int],
                            profileSize: Int, range: Long): Iterator[(Array[Byte], Array[Long], Double)] = {
    if (!it.hasNext) return Iterator.empty
    val ctx = LdgpuNative.context()
    val out = new Array[Long](1)
    LdgpuNative.check(LdgpuNative.countsCreate(ctx, nLangs, grams, 0L, out))
    val counts = out(0)
    try {
      val maxRows = math.max(1L, math.min(range, 1L << 24)).toInt
      val maxKeyBytes = 64 << 20
      val maxPairs = 1 << 24
      val kb = LdgpuNative.direct(maxKeyBytes.toLong)
      val ko = LdgpuNative.direct(8L * (maxRows + 1))
      val po = LdgpuNative.direct(8L * (maxRows + 1))
      val pl = LdgpuNative.direct(4L * maxPairs)
      val pc = LdgpuNative.direct(8L * maxPairs)
      var n = 0
      var keyBytes = 0
      var pairs = 0
      def flush(): Unit = if (n > 0) {
        kb.position(0)
        LdgpuNative.check(LdgpuNative.countsAddSparse(counts, n.toLong, kb, ko, po, pl, pc))
        n = 0
        keyBytes = 0
        pairs = 0
      }
      ko.putLong(0, 0L)
      po.putLong(0, 0L)
      while (it.hasNext) {
        val (key, sc) = it.next()
        val kbytes = key.getBytes(ISO_8859_1)
        if (kbytes.length > maxKeyBytes || sc.langs.length > maxPairs)
          throw new IllegalArgumentException(s"gram of ${kbytes.length} bytes / ${sc.langs.length} languages")
        if (n == maxRows || keyBytes + kbytes.length > maxKeyBytes || pairs + sc.langs.length > maxPairs) flush()
        kb.position(keyBytes)
        kb.put(kbytes)
        keyBytes += kbytes.length
        ko.putLong(8 * (n + 1), keyBytes.toLong)
        var j = 0
        while (j < sc.langs.length) {
          pl.putInt(4 * (pairs + j), sc.langs(j))
          pc.putLong(8 * (pairs + j), sc.counts(j))
          j += 1
        }
        pairs += sc.langs.length
        po.putLong(8 * (n + 1), pairs.toLong)
        n += 1
      }
      flush()
      val size = new Array[Long](2)
      LdgpuNative.check(LdgpuNative.fitTableSize(counts, profileSize, size))
      val (rows, nb) = (size(0), size(1))
      val s = (nLangs + 63) / 64
      val tkb = LdgpuNative.direct(nb)
      val tko = LdgpuNative.direct(8L * (rows + 1))
      val tmk = LdgpuNative.direct(8L * rows * s)
      val tvl = LdgpuNative.direct(8L * rows)
      LdgpuNative.check(LdgpuNative.fitTableExportMasks(counts, tkb, tko, tmk, tvl, rows, nb, nLangs))
      Iterator.tabulate(rows.toInt) { i =>
        val (a, b) = (tko.getLong(8 * i).toInt, tko.getLong(8 * (i + 1)).toInt)
        val key = new Array[Byte](b - a)
        var j = 0
        while (j < key.length) {
          key(j) = tkb.get(a + j)
          j += 1
        }
        val mask = Array.tabulate(s)(w => tmk.getLong(8 * (i * s + w)))
        (key, mask, tvl.getDouble(8 * i))
      }.toArray.iterator
    } finally {
      LdgpuNative.countsDestroy(counts)
    }
  }

  /** (length, unsigned bytes) order: the build's top-K tie rule */
  private val keyOrder: Ordering[Array[Byte]] = new Ordering[Array[Byte]] {
    override def compare(x: Array[Byte], y: Array[Byte]): Int = {
      if (x.length != y.length) return Integer.compare(x.length, y.length)
      var i = 0
      while (i < x.length) {
        val c = Integer.compare(x(i) & 0xff, y(i) & 0xff)
        if (c != 0) return c
        i += 1
      }
      0
    }
  }

  /** filterTopGrams' final step over the partitions' candidates (mask form):
    * per language the K largest values (ties by key order), the union of the
    * picks with their dense rows (the reference's table type).
    *
    * A candidate's value is log(1 + 1/k), k = its language count (the mask's
    * popcount), so a language's order is its presence classes k = 1, 2, ...
    * then the absent candidates (value 0), each class in key order.  One sort
    * by key, a (language, class) histogram, then one pass in key order that
    * takes every candidate above its language's threshold class and the first
    * need(l) of the threshold class (and of the zero-valued fill when a
    * language has fewer than K present candidates): O(C log C + C L) instead
    * of a full sort per language (the device's pair_hist / pair_select rule). */
  private def selectTopK(candidates: Array[(Array[Byte], Array[Long], Double)], nLangs: Int,
                         profileSize: Int): Map[Seq[Byte], Array[Double]] = {
    val K = math.max(profileSize, 0)
    if (K == 0 || candidates.isEmpty) return Map.empty
    val byKey = candidates.sortWith((a, b) => keyOrder.lt(a._1, b._1))
    val C = byKey.length
    val kOf = new Array[Int](C)
    val hist = Array.ofDim[Int](nLangs, nLangs + 2)
    var i = 0
    while (i < C) {
      val m = byKey(i)._2
      var k = 0
      var w = 0
      while (w < m.length) { k += java.lang.Long.bitCount(m(w)); w += 1 }
      kOf(i) = k
      w = 0
      while (w < m.length) {
        var bits = m(w)
        while (bits != 0L) {
          val l = 64 * w + java.lang.Long.numberOfTrailingZeros(bits)
          if (l < nLangs) hist(l)(k) += 1
          bits &= bits - 1
        }
        w += 1
      }
      i += 1
    }
    // per language: threshold class kStar (nLangs + 1: the absent class) and
    // how many of it to take
    val kStar = Array.fill(nLangs)(nLangs + 2)
    val need = new Array[Int](nLangs)
    var fillLangs = List.empty[Int]
    var l = 0
    while (l < nLangs) {
      var acc = 0
      var k = 1
      while (k <= nLangs && kStar(l) == nLangs + 2) {
        if (acc + hist(l)(k) >= K) {
          kStar(l) = k
          need(l) = K - acc
        }
        acc += hist(l)(k)
        k += 1
      }
      if (kStar(l) == nLangs + 2 && K > 0) {  // fewer than K present: every present one, then the fill
        kStar(l) = nLangs + 1
        need(l) = K - acc
        fillLangs = l :: fillLangs
      }
      l += 1
    }
    val taken = new Array[Int](nLangs)
    val chosen = new java.util.BitSet(C)
    i = 0
    while (i < C) {
      val m = byKey(i)._2
      val k = kOf(i)
      var w = 0
      while (w < m.length) {
        var bits = m(w)
        while (bits != 0L) {
          val l = 64 * w + java.lang.Long.numberOfTrailingZeros(bits)
          if (l < nLangs) {
            if (k < kStar(l)) chosen.set(i)
            else if (k == kStar(l) && taken(l) < need(l)) {
              chosen.set(i)
              taken(l) += 1
            }
          }
          bits &= bits - 1
        }
        w += 1
      }
      for (fl <- fillLangs) {  // absent from fl: the zero-valued fill, in key order
        if (((m(fl / 64) >>> (fl % 64)) & 1L) == 0L && taken(fl) < need(fl)) {
          chosen.set(i)
          taken(fl) += 1
        }
      }
      i += 1
    }
    def v(i: Int, l: Int): Double = if (((byKey(i)._2(l / 64) >>> (l % 64)) & 1L) != 0L) byKey(i)._3 else 0.0
    (0 until C).filter(i => chosen.get(i))
      .map(i => (byKey(i)._1.toSeq: Seq[Byte]) -> Array.tabulate(nLangs)(x => v(i, x))).toMap
  }

  def save[T](saveFile: String, ds: Dataset[T]): Unit = {
    logInfo(s"Saving dataset to $saveFile")
    ds.write.format("parquet").mode(SaveMode.Overwrite).save(saveFile)
  }
}
