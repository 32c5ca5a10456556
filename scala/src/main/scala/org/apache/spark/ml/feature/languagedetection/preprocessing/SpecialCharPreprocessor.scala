package org.apache.spark.ml.feature.languagedetection.preprocessing

import org.apache.spark.ml.Transformer
import org.apache.spark.ml.param.ParamMap
import org.apache.spark.ml.param.shared.HasOutputCol
import org.apache.spark.ml.util.{Identifiable, SchemaUtils}
import org.apache.spark.sql.functions.{col, udf}
import org.apache.spark.sql.types.{StringType, StructType}
import org.apache.spark.sql.{DataFrame, Dataset}

/**
 * Host-side drop-in for the reference's SpecialCharPreprocessor
 * (SpecialCharPreprocessor.scala:19-70): same package, class, constructors,
 * param and default (`outputCol` = "fulltext").  Not GPU work.
 *
 * Behaviour kept as the reference has it: `setInputCol` sets `outputCol` (:30);
 * the column is dropped and re-appended last; the text goes through
 * `replaceAll(symbols, "")` then `replaceAll("  *", "")` (:54-56).  The first
 * call hands the symbol list to `String.replaceAll` as a REGEX: it opens a
 * character class that its trailing lone backslash leaves unclosed, so
 * `Pattern.compile` throws `PatternSyntaxException` on the first non-null row
 * (a null text: NullPointerException) -- the reference's transform fails, and so
 * does this one, in the same place.  (The documented intent, symbols removed
 * literally, is `intended_special_char_clean` in the Python mirror.)
 */
class SpecialCharPreprocessor(override val uid: String) extends Transformer with HasOutputCol {

  def this() = this(Identifiable.randomUID("SpecialCharPreprocessor"))

  setDefault(outputCol -> "fulltext")

  /** Sets `outputCol`, as the reference does. */
  def setInputCol(value: String): this.type = set(outputCol, value)

  override def copy(extra: ParamMap): Transformer = defaultCopy(extra)

  override def transformSchema(schema: StructType): StructType =
    SchemaUtils.appendColumn(StructType(schema.fields.filterNot(_.name == $(outputCol))), $(outputCol), StringType,
      nullable = true)

  override def transform(dataset: Dataset[_]): DataFrame = {
    val text = $(outputCol)
    val cleaned = udf { (s: String) =>
      s.replaceAll(SpecialCharPreprocessor.Symbols, "").replaceAll(SpecialCharPreprocessor.Spaces, "")
    }
    val df = dataset.toDF()
    df.schema.fieldIndex(text)
    val tmp = LowerCasePreprocessor.freshName(df, text)
    df.withColumn(tmp, cleaned(col(text))).drop(text).withColumnRenamed(tmp, text)
  }
}

object SpecialCharPreprocessor {
  /** The reference's first replaceAll argument (SpecialCharPreprocessor.scala:55), used as a regex. */
  val Symbols: String = "/_[]*()%^&@$#:|{}<>~`\"\\"
  /** The second (:56): a space and any further spaces. */
  val Spaces: String = "  *"
}
