rule short {
 strings:
  $a = "a"
  $b = { 00 01 }
  $c = "xyz"
  $d = "abcd"
  $e = "bcd"
  $f = { FF FF FF FF }
  $g = "Hello" wide
  $h = "AbC" nocase
  $i = "aaaa"
  $j = "aaa"
 condition: any of them
}
