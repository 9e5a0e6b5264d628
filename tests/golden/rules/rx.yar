rule rx_text {
 strings:
  $a = /https?:\/\/[a-z0-9]{3,10}\.com/
  $b = /Content-Type: [a-z]+\/[a-z]+/ nocase
  $c = /username(_id)?=[A-Za-z0-9_]{4,}/
  $d = /\bpassword\b/ wide ascii
  $e = /GET \/[a-z]+\.php\?id=[0-9]+/
  $f = /abcde.{2,5}vwxyz/s
  $g = /(cat|dog|bird)house/
  $h = /Qx[^\n]{2,8}Zq!/
 condition: any of them
}
rule rx_hex_alt {
 strings:
  $a = { 4D 5A ( 90 00 | 50 00 ) 03 [2-4] FF FF }
  $b = { E8 ?? ?? ?? ?? ( 5B | 5D ) C3 }
  $c = { 11 22 33 44 ( 55 | 66 77 | 88 99 AA ) BB }
 condition: any of them
}
