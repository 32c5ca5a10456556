package org.apache.spark.ml.feature.languagedetection.preprocessing

import java.nio.ByteBuffer
import java.util.Locale

import org.apache.spark.ml.feature.languagedetection.LdgpuNative

/**
 * The preprocessors of a batch of documents on the executor's GPU
 * (ldgpu_preprocess, include/ldgpu.h PREPROCESS): lower-casing in the locale of
 * each document's label (LowerCasePreprocessor.scala:60) and the symbol /
 * space cleanup (SpecialCharPreprocessor.scala:55-56, its documented intent).
 *
 * The device's case map is built from THIS JVM (Character.toLowerCase of
 * every UTF-16 unit; `special` = the units whose String.toLowerCase is not
 * that 1:1 mapping), so the device lower-cases as the executor's own JVM
 * does.  Documents the device cannot lower-case 1:1 (host flag) are
 * lower-cased here with String.toLowerCase, then cleaned like the device does.
 */
object DevicePreprocess {

  @volatile private var map: Long = 0L

  private def caseMap(): Long = {
    if (map == 0L) synchronized {
      if (map == 0L) {
        val lower = LdgpuNative.direct(2L * 65536)
        val special = new Array[Byte](8192)
        var u = 0
        while (u < 65536) {
          val c = u.toChar
          if (Character.isSurrogate(c)) {
            lower.putShort(2 * u, u.toShort)
          } else {
            val low = String.valueOf(c).toLowerCase(Locale.ROOT)
            if (low.length == 1) lower.putShort(2 * u, low.charAt(0).toShort)
            else {
              lower.putShort(2 * u, u.toShort)
              special(u >> 3) = (special(u >> 3) | (1 << (u & 7))).toByte
            }
          }
          u += 1
        }
        // capital sigma: Final_Sigma depends on the context
        special(0x3A3 >> 3) = (special(0x3A3 >> 3) | (1 << (0x3A3 & 7))).toByte
        // high surrogates of the supplementary planes holding cased letters
        var cp = 0x10000
        while (cp < 0x110000) {
          if (Character.toLowerCase(cp) != cp) {
            val hi = 0xD800 + ((cp - 0x10000) >> 10)
            special(hi >> 3) = (special(hi >> 3) | (1 << (hi & 7))).toByte
          }
          cp += 1
        }
        val sp = LdgpuNative.direct(8192)
        sp.put(special)
        val out = new Array[Long](1)
        LdgpuNative.check(LdgpuNative.casemapCreate(LdgpuNative.context(), lower, sp, out))
        map = out(0)
      }
    }
    map
  }

  /** the locale class of a label (Locale.forLanguageTag(lang).getLanguage) */
  def localeClass(lang: String): Byte = Locale.forLanguageTag(lang).getLanguage match {
    case "tr" | "az" => LdgpuNative.LocaleTrAz.toByte
    case "lt" => LdgpuNative.LocaleLt.toByte
    case _ => LdgpuNative.LocaleRoot.toByte
  }

  private val symbols = "/_[]*()%^&@$#:|{}<>~`\"\\ "

  private def clean(s: String): String = s.filterNot(c => symbols.indexOf(c) >= 0)

  /**
   * The batch through the device.  lower: each text lower-cased in the locale
   * of its label (a null text or label: NullPointerException, as the
   * reference's row map); clean: the symbols and spaces removed.
   */
  def run(texts: Array[String], langs: Array[String], lower: Boolean, clean: Boolean): Array[String] = {
    val n = texts.length
    val offsets = LdgpuNative.direct(8L * (n + 1))
    var units = 0L
    var i = 0
    while (i < n) {
      offsets.putLong(8 * i, units)
      units += texts(i).length           // NullPointerException on a null text
      i += 1
    }
    offsets.putLong(8 * n, units)
    val in = LdgpuNative.direct(2L * units)
    val locale = if (lower) LdgpuNative.direct(n.toLong) else null
    i = 0
    while (i < n) {
      val t = texts(i)
      val at = offsets.getLong(8 * i).toInt
      var k = 0
      while (k < t.length) { in.putShort(2 * (at + k), t.charAt(k).toShort); k += 1 }
      if (lower) locale.put(i, localeClass(langs(i)))  // NullPointerException on a null label
      i += 1
    }
    val flags = (if (lower) LdgpuNative.PreLower else 0) | (if (clean) LdgpuNative.PreClean else 0)
    val out = LdgpuNative.direct(2L * units)
    val outOffsets = LdgpuNative.direct(8L * (n + 1))
    val host = LdgpuNative.direct(n.toLong)
    LdgpuNative.check(LdgpuNative.preprocess(caseMap(), in, offsets, n.toLong, locale, flags, out, outOffsets, host))
    val res = new Array[String](n)
    i = 0
    while (i < n) {
      if (host.get(i) != 0) {
        val low = if (lower) texts(i).toLowerCase(Locale.forLanguageTag(langs(i))) else texts(i)
        res(i) = if (clean) DevicePreprocess.clean(low) else low
      } else {
        val b = outOffsets.getLong(8 * i).toInt
        val e = outOffsets.getLong(8 * (i + 1)).toInt
        val cs = new Array[Char](e - b)
        var k = 0
        while (k < cs.length) { cs(k) = out.getShort(2 * (b + k)).toChar; k += 1 }
        res(i) = new String(cs)
      }
      i += 1
    }
    res
  }
}
