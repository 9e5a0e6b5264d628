/*
    Add padding for making the file large enough to trigger issue #884

    pading pading pading pading pading pading pading pading pading pading
    pading pading pading pading pading pading pading pading pading pading
    pading pading pading pading pading pading pading pading pading pading
    pading pading pading pading pading pading pading pading pading pading
    pading pading pading pading pading pading pading pading pading pading
    pading pading pading pading pading pading pading pading pading pading
    pading pading pading pading pading pading pading pading pading pading
    pading pading pading pading pading pading pading pading pading pading
    pading pading pading pading pading pading pading pading pading pading
    pading pading pading pading pading pading pading pading pading pading
    pading pading pading pading pading pading pading pading pading pading
    pading pading pading pading pading pading pading pading pading pading
    pading pading pading pading pading pading pading pading pading pading
    pading pading pading pading pading pading pading pading pading pading
    pading pading pading pading pading pading pading pading pading pading
    pading pading pading pading pading pading pading pading pading pading
    pading pading pading pading pading pading pading pading pading pading
    pading pading pading pading pading pading pading pading pading pading
*/

rule baz { condition: true }
