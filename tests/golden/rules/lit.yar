rule lit_plain {
 strings:
  $a = "HelloWorld"
  $b = "xyzzy1234"
  $c = "ab"
  $d = "Quartz"
 condition: any of them
}
rule lit_wide {
 strings:
  $a = "WideString" wide
  $b = "AsciiAndWide" ascii wide
 condition: any of them
}
rule lit_nocase {
 strings:
  $a = "CaseLess" nocase
  $b = "NoCaseWide" nocase wide ascii
  $c = "zz" nocase
 condition: any of them
}
rule lit_xor {
 strings:
  $a = "XorMe!" xor
  $b = "XorWide" xor wide
  $c = "XorRange" xor(1-16)
 condition: any of them
}
rule lit_fixed {
 strings:
  $a = "FixedHere"
 condition: $a at 4096
}
rule lit_fullword {
 strings:
  $a = "word" fullword
 condition: $a
}
rule lit_private {
 strings:
  $a = "secretstr" private
 condition: $a
}
rule lit_base64 {
 strings:
  $a = "base64text" base64
 condition: $a
}
rule hex_mix {
 strings:
  $a = { 41 42 43 44 45 46 }
  $b = { 61 62 ?? 64 65 }
  $c = { 31 32 33 [2-4] 37 38 }
 condition: any of them
}
