package org.apache.spark.ml.feature.languagedetection.language

/**
 * The reference's language enumeration (Language.scala:11-200), same package,
 * object name and public members: `isoLanguageCodes` (ISO 639-1, in the
 * reference's order) and one enumeration value per code whose id is its
 * position.  It is not on the GPU path -- `LanguageDetector` and
 * `LanguageDetectorModel` take a plain `Seq[String]` of languages, as in the
 * reference -- and is kept so callers of the reference find it.
 */
object Language extends Enumeration {

  /** ISO 639-1 codes; the value of code i has id i. */
  val isoLanguageCodes: Seq[String] = (
    "ab aa af ak sq am ar an hy as av ae ay az bm ba eu be bn bh bi bs br bg my ca km ch ce ny zh " +
    "cu cv kw co cr hr cs da dv nl dz en eo et ee fj fi fr ff gd gl lg ka de ki el kl gn gu ht ha " +
    "he hz hi ho hu is io ig id ia ie iu ik ga it ja jv kn kr ks kk rw kv kg ko kj ku ky lo la lv " +
    "lb li ln lt lu mk mg ms ml mt gv mi mr mh ro mn na nv nd ng ne se no nb nn ii oc oj or om os " +
    "pi pa ps fa pl pt qu rm rn ru sm sg sa sc sr sn sd si sk sl so st nr es su sw ss sv tl ty tg " +
    "ta tt te th bo ti to ts tn tr tk tw uk ur uz ve vi vo wa cy fy wo xh yi yo za zu"
  ).split(' ').toSeq

  for ((code, id) <- isoLanguageCodes.zipWithIndex) Value(id, code)
}
