"""Character text front end for Synthesizer.tts.

Restates the reference's character path: `TTS/tts/utils/text/symbols.py` (make_symbols and the
default symbol set), `TTS/tts/utils/text/__init__.py:117-190` (text_to_sequence with {ARPAbet}
spans, _should_keep_symbol) and `TTS/tts/utils/text/cleaners.py` (the cleaner pipelines).

Third-party pieces of the reference front end are absent from this image and are replaced:
  * `unidecode` (convert_to_ascii): NFKD decomposition with non-ASCII marks dropped. Identical
    for accented Latin letters, different for symbols unidecode spells out.
  * `inflect` (number_norm.py): `number_to_words` below restates inflect's English output for
    the call forms number_norm.py uses (andword='', group=2 years, ordinals).
  * `phonemizer` / espeak (phoneme_to_sequence): not restated; phoneme configs need a caller
    supplied `phonemize(text, language) -> str` (same "|"-separated format as text2phone).
The symbol tables are pinned against the reference (tests/golden/text_symbols.json); the
number and transliteration substitutes are parity-unpinned (their references are not importable).
"""
import re
import unicodedata

_pad, _eos, _bos = "_", "~", "^"
_characters = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz!'(),-.:;? "
_punctuations = "!'(),-.:;? "
_phoneme_punctuations = ".!;:,?"
_vowels = "iyɨʉɯuɪʏʊeøɘəɵɤoɛœɜɞʌɔæɐaɶɑɒᵻ"
_non_pulmonic_consonants = "ʘɓǀɗǃʄǂɠǁʛ"
_pulmonic_consonants = "pbtdʈɖcɟkɡqɢʔɴŋɲɳnɱmʙrʀⱱɾɽɸβfvθðszʃʒʂʐçʝxɣχʁħʕhɦɬɮʋɹɻjɰlɭʎʟ"
_suprasegmentals = "ˈˌːˑ"
_other_symbols = "ʍwɥʜʢʡɕʑɺɧ"
_diacrilics = "ɚ˞ɫ"
_phonemes = (_vowels + _non_pulmonic_consonants + _pulmonic_consonants + _suprasegmentals + _other_symbols
             + _diacrilics)


def make_symbols(characters, phonemes, punctuations="!'(),-.:;? ", pad="_", eos="~", bos="^"):
    """symbols.py:8-20: [pad, eos, bos] + characters + '@'ARPAbet; phonemes sorted + punctuations."""
    ph_sorted = sorted(list(phonemes))
    arpabet = ["@" + s for s in ph_sorted]
    return [pad, eos, bos] + list(characters) + arpabet, [pad, eos, bos] + ph_sorted + list(punctuations)


symbols, phonemes = make_symbols(_characters, _phonemes, _punctuations, _pad, _eos, _bos)

# ------------------------------------------------------------------ numbers (inflect stand-in)
_ONES = ["zero", "one", "two", "three", "four", "five", "six", "seven", "eight", "nine", "ten", "eleven",
         "twelve", "thirteen", "fourteen", "fifteen", "sixteen", "seventeen", "eighteen", "nineteen"]
_TENS = ["", "", "twenty", "thirty", "forty", "fifty", "sixty", "seventy", "eighty", "ninety"]
_SCALES = ["", "thousand", "million", "billion", "trillion", "quadrillion"]
_ORD = {"one": "first", "two": "second", "three": "third", "five": "fifth", "eight": "eighth", "nine": "ninth",
        "twelve": "twelfth"}


def _two(n):
    return _ONES[n] if n < 20 else _TENS[n // 10] + ("-" + _ONES[n % 10] if n % 10 else "")


def _three(n):
    h, r = divmod(n, 100)
    parts = ([_ONES[h] + " hundred"] if h else []) + ([_two(r)] if r else [])
    return " ".join(parts)


def number_to_words(n, group=0, zero="zero"):
    """inflect.engine().number_to_words(n, andword='') (group=0) and (..., zero='oh', group=2)."""
    n = int(n)
    if group == 2:
        s = str(n)
        if len(s) % 2:
            s = "0" + s if len(s) > 1 else s
        out = []
        for i in range(0, len(s), 2):
            pair = int(s[i:i + 2])
            if s[i] == "0" and i + 1 < len(s):
                out.append(zero + (" " + _ONES[int(s[i + 1])] if s[i + 1] != "0" else " " + zero))
            else:
                out.append(_two(pair))
        return ", ".join(out)
    if n == 0:
        return zero
    groups = []
    while n:
        n, g = divmod(n, 1000)
        groups.append(g)
    words = [(_three(g) + (" " + _SCALES[i] if _SCALES[i] else "")) for i, g in enumerate(groups) if g]
    return ", ".join(reversed(words))


def _ordinal(words):
    last = re.split(r"([ -])", words)
    w = last[-1]
    if w in _ORD:
        w = _ORD[w]
    elif w.endswith("y"):
        w = w[:-1] + "ieth"
    else:
        w = w + "th"
    return "".join(last[:-1]) + w


_comma_number_re = re.compile(r"([0-9][0-9\,]+[0-9])")
_decimal_number_re = re.compile(r"([0-9]+\.[0-9]+)")
_pounds_re = re.compile(r"£([0-9\,]*[0-9]+)")
_dollars_re = re.compile(r"\$([0-9\.\,]*[0-9]+)")
_ordinal_re = re.compile(r"[0-9]+(st|nd|rd|th)")
_number_re = re.compile(r"[0-9]+")


def _expand_dollars(m):
    """number_norm.py:23-41"""
    match = m.group(1)
    parts = match.split(".")
    if len(parts) > 2:
        return match + " dollars"
    dollars = int(parts[0]) if parts[0] else 0
    cents = int(parts[1]) if len(parts) > 1 and parts[1] else 0
    if dollars and cents:
        return "%s %s, %s %s" % (dollars, "dollar" if dollars == 1 else "dollars", cents,
                                 "cent" if cents == 1 else "cents")
    if dollars:
        return "%s %s" % (dollars, "dollar" if dollars == 1 else "dollars")
    if cents:
        return "%s %s" % (cents, "cent" if cents == 1 else "cents")
    return "zero dollars"


def _expand_number(m):
    """number_norm.py:48-61"""
    num = int(m.group(0))
    if 1000 < num < 3000:
        if num == 2000:
            return "two thousand"
        if 2000 < num < 2010:
            return "two thousand " + number_to_words(num % 100)
        if num % 100 == 0:
            return number_to_words(num // 100) + " hundred"
        return number_to_words(num, group=2, zero="oh").replace(", ", " ")
    return number_to_words(num)


def normalize_numbers(text):
    """number_norm.py:64-71"""
    text = re.sub(_comma_number_re, lambda m: m.group(1).replace(",", ""), text)
    text = re.sub(_pounds_re, r"\1 pounds", text)
    text = re.sub(_dollars_re, _expand_dollars, text)
    text = re.sub(_decimal_number_re, lambda m: m.group(1).replace(".", " point "), text)
    text = re.sub(_ordinal_re, lambda m: _ordinal(number_to_words(int(m.group(0)[:-2]))), text)
    text = re.sub(_number_re, _expand_number, text)
    return text


# ------------------------------------------------------------------ cleaners (cleaners.py)
_whitespace_re = re.compile(r"\s+")
_abbreviations_en = [(re.compile("\\b%s\\." % a, re.IGNORECASE), b) for a, b in [
    ("mrs", "misess"), ("mr", "mister"), ("dr", "doctor"), ("st", "saint"), ("co", "company"), ("jr", "junior"),
    ("maj", "major"), ("gen", "general"), ("drs", "doctors"), ("rev", "reverend"), ("lt", "lieutenant"),
    ("hon", "honorable"), ("sgt", "sergeant"), ("capt", "captain"), ("esq", "esquire"), ("ltd", "limited"),
    ("col", "colonel"), ("ft", "fort")]]


def convert_to_ascii(text):
    return unicodedata.normalize("NFKD", text).encode("ascii", "ignore").decode("ascii")


def collapse_whitespace(text):
    return re.sub(_whitespace_re, " ", text).strip()


def expand_abbreviations(text):
    for regex, rep in _abbreviations_en:
        text = re.sub(regex, rep, text)
    return text


def replace_symbols(text):
    return text.replace(";", ",").replace("-", " ").replace(":", ",").replace("&", " and ")


def remove_aux_symbols(text):
    return re.sub(r"[\<\>\(\)\[\]\"]+", "", text)


def basic_cleaners(text):
    return collapse_whitespace(text.lower())


def transliteration_cleaners(text):
    return collapse_whitespace(convert_to_ascii(text).lower())


def english_cleaners(text):
    text = convert_to_ascii(text).lower()
    text = normalize_numbers(text)
    text = expand_abbreviations(text)
    text = replace_symbols(text)
    text = remove_aux_symbols(text)
    return collapse_whitespace(text)


def phoneme_cleaners(text):
    text = convert_to_ascii(text)
    text = normalize_numbers(text)
    text = expand_abbreviations(text)
    text = replace_symbols(text)
    text = remove_aux_symbols(text)
    return collapse_whitespace(text)


CLEANERS = {f.__name__: f for f in (basic_cleaners, transliteration_cleaners, english_cleaners, phoneme_cleaners)}
_CURLY_RE = re.compile(r"(.*?)\{(.+?)\}(.*)")


def _clean(text, cleaner_names):
    for name in cleaner_names:
        if name not in CLEANERS:
            raise NotImplementedError(f"text cleaner '{name}' is not restated in this build")
        text = CLEANERS[name](text)
    return text


def text_to_sequence(text, cleaner_names, tp=None):
    """text/__init__.py:117-140: ids of the cleaned text, {ARPAbet} spans as '@' symbols."""
    syms = make_symbols(**tp)[0] if tp else symbols
    s2i = {s: i for i, s in enumerate(syms)}

    def keep(seq):
        return [s2i[s] for s in seq if s in s2i and s not in ("~", "^", "_")]

    seq = []
    while text:
        m = _CURLY_RE.match(text)
        if not m:
            seq += keep(_clean(text, cleaner_names))
            break
        seq += keep(_clean(m.group(1), cleaner_names))
        seq += keep(["@" + s for s in m.group(2).split()])
        text = m.group(3)
    return seq


def phoneme_to_sequence(text, cleaner_names, language, enable_eos_bos=False, tp=None, phonemize=None):
    """text/__init__.py:84-101 with a caller-supplied phonemizer (espeak is not in this image)."""
    if phonemize is None:
        raise NotImplementedError("phoneme input needs phonemizer/espeak, which this image lacks; "
                                  "pass phonemize=callable(text, language) -> '|'-separated phonemes")
    ph = make_symbols(**tp)[1] if tp else phonemes
    p2i = {s: i for i, s in enumerate(ph)}
    seq = []
    for p in filter(None, phonemize(_clean(text, cleaner_names), language).split("|")):
        seq += [p2i[s] for s in p if s in p2i and s not in ("~", "^", "_")]
    if enable_eos_bos:
        seq = [p2i[tp["bos"] if tp else _bos]] + seq + [p2i[tp["eos"] if tp else _eos]]
    return seq


def text_to_seqvec(text, config, phonemize=None):
    """synthesis.py:10-22"""
    import numpy as np
    tp = config.get("characters") if hasattr(config, "get") else None
    cleaners = [config["text_cleaner"]]
    if config.get("use_phonemes", False):
        return np.asarray(phoneme_to_sequence(text, cleaners, config.get("phoneme_language", "en-us"),
                                              config.get("enable_eos_bos_chars", False), tp, phonemize), np.int32)
    return np.asarray(text_to_sequence(text, cleaners, tp), np.int32)


def split_into_sentences(text):
    """Stand-in for pysbd.Segmenter(language='en', clean=True).segment (synthesizer.py:131-132;
    pysbd is not in this image): split after . ! ? (plus closing quotes) before whitespace."""
    text = collapse_whitespace(text)
    parts = re.split(r"(?<=[.!?])[\"')\]]*\s+", text)
    return [p.strip() for p in parts if p.strip()]
