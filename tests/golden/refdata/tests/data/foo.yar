include "include/bar.yar"

rule foo { condition: bar }
