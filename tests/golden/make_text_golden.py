"""Writes tests/golden/text_symbols.json from the reference's symbol tables.

Loads /root/reference/TTS/tts/utils/text/symbols.py by file path (the package __init__ imports
phonemizer, which this image lacks; symbols.py itself has no imports). Run in the build
container: python tests/golden/make_text_golden.py
"""
import importlib.util
import json
import os

REF = "/root/reference/TTS/tts/utils/text/symbols.py"
spec = importlib.util.spec_from_file_location("ref_symbols", REF)
mod = importlib.util.module_from_spec(spec)
spec.loader.exec_module(mod)
custom = mod.make_symbols("abc", "xyz", punctuations="!.", pad="P", eos="E", bos="B")
out = {"source": "TTS/tts/utils/text/symbols.py", "symbols": mod.symbols, "phonemes": mod.phonemes,
       "custom_make_symbols": {"args": ["abc", "xyz", "!.", "P", "E", "B"], "symbols": custom[0],
                               "phonemes": custom[1]}}
with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "text_symbols.json"), "w") as f:
    json.dump(out, f, ensure_ascii=False, indent=0)
print(len(mod.symbols), len(mod.phonemes))
