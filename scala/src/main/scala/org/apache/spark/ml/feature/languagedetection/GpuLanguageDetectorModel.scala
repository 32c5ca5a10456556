package org.apache.spark.ml.feature.languagedetection

import org.apache.hadoop.fs.Path
import org.apache.spark.internal.Logging
import org.apache.spark.ml.Model
import org.apache.spark.ml.param.ParamMap
import org.apache.spark.ml.param.shared.{HasInputCol, HasOutputCol}
import org.apache.spark.ml.util._
import org.apache.spark.TaskContext
import org.apache.spark.sql.catalyst.InternalRow
import org.apache.spark.sql.catalyst.expressions.{GenericInternalRow, JoinedRow, UnsafeProjection}
import org.apache.spark.sql.types.{StringType, StructType}
import org.apache.spark.sql.{DataFrame, Dataset, LdgpuSqlBridge, SaveMode}
import org.apache.spark.unsafe.types.UTF8String
import org.json4s.JsonDSL._
import org.json4s.{DefaultFormats, JArray, JString}

/**
  * Drop-in for the reference's LanguageDetectorModel (same package, class
  * name, constructors, public vals -- including the `gramLenghts` spelling --
  * params and defaults; LanguageDetectorModel.scala:168-243).  Scoring runs on
  * the executor's GPU through libldgpu.so: transform broadcasts the table once
  * as flat arrays, and every partition is packed into pinned direct buffers
  * and scored in batches (ldgpu_score), instead of one Scala detect call per
  * row.  Labels and scores are the reference's: the library reproduces the
  * fp64 left fold of BLAS.axpy and breeze's first-maximum argmax.
  */
class LanguageDetectorModel(override val uid: String,
                            val gramProbabilities: Map[Seq[Byte], Array[Double]],
                            val gramLenghts: Seq[Int],
                            val supportedLanguages: Seq[String])
  extends Model[LanguageDetectorModel] with HasInputCol with HasOutputCol with Logging with MLWritable {

  def this(gramProbabilities: Map[Seq[Byte], Array[Double]], gramLengths: Seq[Int], languages: Seq[String]) =
    this(Identifiable.randomUID("LanguageDetectorModel"), gramProbabilities, gramLengths, languages)

  setDefault(inputCol -> "fulltext", outputCol -> "lang")

  def setInputCol(value: String): this.type = set(inputCol, value)
  def setOutputCol(value: String): this.type = set(outputCol, value)

  /** documents and bytes per ldgpu_score call (one pipelined call per batch) */
  var batchDocs: Int = 1 << 20
  var batchBytes: Int = 64 << 20

  override def transformSchema(schema: StructType): StructType = {
    val inputType = schema($(inputCol)).dataType
    require(inputType.sameType(StringType), s"Input type must be StringType but got $inputType.")
    SchemaUtils.appendColumn(schema, $(outputCol), StringType, nullable = true)
  }

  override def copy(extra: ParamMap): LanguageDetectorModel = {
    val m = new LanguageDetectorModel(uid, gramProbabilities, gramLenghts, supportedLanguages)
    copyValues(m, extra).setParent(parent)
  }

  /**
    * transform (LanguageDetectorModel.scala:219-240) on the executor's GPU:
    * the table is broadcast once in packed form (mask form for fit-produced
    * tables), each partition's rows are read as catalyst rows -- the text as
    * Spark's own UTF-8 bytes, copied as they are when ASCII (then UTF-8 IS the
    * reference's low-byte encoding, :161), decoded and low-byte encoded
    * otherwise -- packed into pinned buffers and scored in batches
    * (ldgpu_score), and the label is appended to every row.  The device table
    * and the pinned buffers are released when the task completes, also when
    * the iterator is not drained (limit, show, a failed task).
    */
  override def transform(dataset: Dataset[_]): DataFrame = {
    val schema = transformSchema(dataset.schema)
    val spark = dataset.sparkSession
    val table = spark.sparkContext.broadcast(PackedTable.of(gramProbabilities, supportedLanguages.length))
    val grams = gramLenghts.toArray
    val nLangs = supportedLanguages.length
    val labels = supportedLanguages.map(l => UTF8String.fromString(l)).toArray
    val idx = dataset.schema.fieldIndex($(inputCol))
    val nDocs = batchDocs
    val nBytes = batchBytes
    val df = dataset.toDF()
    val rows = LdgpuSqlBridge.internalRows(df).mapPartitions { it =>
      if (!it.hasNext) Iterator.empty
      else {
        val model = LdgpuNative.acquireModel(table.id, table.value, grams)
        val batch = new DocBatch(LdgpuNative.context(), nDocs, nBytes)
        val task = TaskContext.get()
        if (task != null) task.addTaskCompletionListener { _: TaskContext =>
          batch.close()
          LdgpuNative.releaseModel(table.id)
        }
        val pending = new java.util.ArrayList[InternalRow](math.min(nDocs, 1 << 16))
        val project = UnsafeProjection.create(schema)
        new Iterator[InternalRow] {
          private var out: Iterator[InternalRow] = Iterator.empty
          // the next batch of rows: packed, scored in one ldgpu_score call
          private def fill(): Unit = {
            batch.clear()
            pending.clear()
            while (it.hasNext && !batch.full) {
              val row = it.next()
              val text = row.getUTF8String(idx)
              if (text == null) throw new NullPointerException(s"null text in column ${schema(idx).name}")
              batch.addScoreUtf8(text.getBaseObject, text.getBaseOffset, text.numBytes, text.toString)
              pending.add(row.copy())  // the child iterator may reuse its row object
            }
            LdgpuNative.check(
              LdgpuNative.score(model, batch.bytes, batch.offsets, batch.n.toLong, batch.labels, null, nLangs))
            val scored = new Array[InternalRow](batch.n)
            var i = 0
            while (i < batch.n) {
              val label = new GenericInternalRow(Array[Any](labels(batch.label(i))))
              scored(i) = project(new JoinedRow(pending.get(i), label)).copy()
              i += 1
            }
            out = scored.iterator
          }
          override def hasNext: Boolean = {
            if (!out.hasNext && it.hasNext) fill()
            out.hasNext
          }
          override def next(): InternalRow = {
            if (!hasNext) throw new NoSuchElementException
            out.next()
          }
        }
      }
    }
    LdgpuSqlBridge.fromInternalRows(spark, rows, schema)
  }

  override def write: MLWriter = new LanguageDetectorModel.LanguageDetectorModelWriter(this)
}

object LanguageDetectorModel extends MLReadable[LanguageDetectorModel] {

  override def read: MLReader[LanguageDetectorModel] = new LanguageDetectorModelReader
  override def load(path: String): LanguageDetectorModel = super.load(path)

  /**
    * detect(Array[Byte], ...) (LanguageDetectorModel.scala:131-156): one
    * document.  The reference's callers put detect in a UDF, calling it per
    * row with the same map, so the device table of a map is kept.  The
    * reference reads the map on every call, and a Map's Array[Double] values
    * can be edited in place, so a kept table serves a call only while the
    * map is the same object (eq) AND its rows equal (bitwise) a copy taken
    * when the table was built (unchanged: one Arrays.equals per row).  The last
    * `detectCacheSize` tables stay resident (reference-counted: an evicted
    * table is destroyed once no call is scoring with it); each thread keeps
    * its own direct buffers.  For many documents, transform scores in
    * batches.
    */
  def detect(text: Array[Byte], probabilityMap: Map[Seq[Byte], Array[Double]], supportedLanguages: Seq[String],
             gramLengths: Seq[Int]): String = {
    val e = detectAcquire(probabilityMap, supportedLanguages.length, gramLengths)
    try {
      val b = detectBuffers.get().ensure(text.length)
      b.bytes.clear()
      b.bytes.put(text).flip()
      b.offsets.putLong(0, 0L)
      b.offsets.putLong(8, text.length.toLong)
      LdgpuNative.check(LdgpuNative.score(e.model, b.bytes, b.offsets, 1L, b.label, null, supportedLanguages.length))
      supportedLanguages(b.label.getInt(0))
    } finally {
      detectRelease(e)
    }
  }

  var detectCacheSize: Int = 4

  private final class DetectEntry(val map: AnyRef, val snapshot: Map[Seq[Byte], Array[Double]], val grams: Seq[Int],
                                   val nLangs: Int, val model: Long) {
    var refs = 0
    var evicted = false
  }
  private val detectCache = new java.util.ArrayDeque[DetectEntry]()

  private def detectAcquire(map: Map[Seq[Byte], Array[Double]], nLangs: Int, grams: Seq[Int]): DetectEntry =
    detectCache.synchronized {
      val it = detectCache.iterator()
      while (it.hasNext) {
        val e = it.next()
        if ((e.map eq map) && e.nLangs == nLangs && e.grams == grams && unchanged(map, e.snapshot)) {
          e.refs += 1
          return e
        }
      }
      val model = PackedTable.of(map, nLangs).upload(LdgpuNative.context(), grams.toArray)
      val e = new DetectEntry(map, map.map { case (k, v) => (k, v.clone()) }, grams.toList, nLangs, model)
      e.refs = 1
      detectCache.addFirst(e)
      while (detectCache.size > math.max(1, detectCacheSize)) {
        val old = detectCache.removeLast()
        old.evicted = true
        if (old.refs == 0) LdgpuNative.modelDestroy(old.model)
      }
      e
    }

  /** every row of map equals (bitwise, java.util.Arrays.equals) the snapshot's */
  private def unchanged(map: Map[Seq[Byte], Array[Double]], snap: Map[Seq[Byte], Array[Double]]): Boolean =
    map.size == snap.size && map.forall { case (k, v) =>
      snap.get(k) match {
        case Some(w) => java.util.Arrays.equals(v, w)
        case None => false
      }
    }

  private def detectRelease(e: DetectEntry): Unit = detectCache.synchronized {
    e.refs -= 1
    if (e.evicted && e.refs == 0) LdgpuNative.modelDestroy(e.model)
  }

  /** a thread's direct buffers of one document (grown as documents grow) */
  private final class DetectBuffers {
    var bytes: java.nio.ByteBuffer = LdgpuNative.direct(4096)
    val offsets: java.nio.ByteBuffer = LdgpuNative.direct(16)
    val label: java.nio.ByteBuffer = LdgpuNative.direct(4)
    def ensure(n: Int): DetectBuffers = {
      if (bytes.capacity < n + 16) bytes = LdgpuNative.direct(math.max(2L * bytes.capacity, n + 16L))
      this
    }
  }
  private val detectBuffers = new ThreadLocal[DetectBuffers] {
    override def initialValue(): DetectBuffers = new DetectBuffers
  }

  /** detect(String, ...) (:158-165): the low byte of every UTF-16 unit */
  def detect(text: String, probabilityMap: Map[Seq[Byte], Array[Double]], supportedLanguages: Seq[String],
             gramLengths: Seq[Int]): String =
    detect(text.toCharArray.map(_.toByte), probabilityMap, supportedLanguages, gramLengths)

  /**
    * The reference's on-disk layout (:27-60): metadata JSON, probabilities
    * (_1 array<tinyint>, _2 array<double>), supportedLanguages and gramLengths
    * (`value`).  The metadata also carries "languageOrder": the reference's
    * reader collects supportedLanguages without an ordering key (:82-87), so a
    * multi-part dataset can come back permuted; this reader uses the pin, the
    * reference's reader ignores the extra top-level field.
    */
  class LanguageDetectorModelWriter(instance: LanguageDetectorModel) extends MLWriter with Logging {
    override protected def saveImpl(path: String): Unit = {
      val spark = sparkSession
      import spark.implicits._
      DefaultParamsWriter.saveMetadata(instance, path, sc,
        extraMetadata = Some("languageOrder" -> instance.supportedLanguages.toList))
      spark.createDataset(instance.gramProbabilities.toSeq).write.mode(SaveMode.Overwrite)
        .parquet(new Path(path, "probabilities").toString)
      spark.createDataset(instance.supportedLanguages).coalesce(1).write.mode(SaveMode.Overwrite)
        .parquet(new Path(path, "supportedLanguages").toString)
      spark.createDataset(instance.gramLenghts).coalesce(1).write.mode(SaveMode.Overwrite)
        .parquet(new Path(path, "gramLengths").toString)
    }
  }

  class LanguageDetectorModelReader extends MLReader[LanguageDetectorModel] {
    private val className = classOf[LanguageDetectorModel].getName

    override def load(path: String): LanguageDetectorModel = {
      val spark = sparkSession
      import spark.implicits._
      val metadata = DefaultParamsReader.loadMetadata(path, sc, className)
      val probabilities = spark.read.parquet(new Path(path, "probabilities").toString)
        .as[(Seq[Byte], Array[Double])].collect().toMap
      val stored = spark.read.parquet(new Path(path, "supportedLanguages").toString).as[String].collect().toSeq
      implicit val formats: DefaultFormats.type = DefaultFormats
      val languages = metadata.metadata \ "languageOrder" match {
        case JArray(values) =>
          val pinned = values.collect { case JString(s) => s }
          require(pinned.sorted == stored.sorted,
            s"metadata languageOrder $pinned does not match the supportedLanguages dataset $stored")
          pinned
        case _ => stored
      }
      val grams = spark.read.parquet(new Path(path, "gramLengths").toString).as[Int].collect().toSeq
      val model = new LanguageDetectorModel(metadata.uid, probabilities, grams, languages)
      DefaultParamsReader.getAndSetParams(model, metadata)
      model
    }
  }
}
